#!/usr/bin/env python3
"""EDNet detection training (the reference's real caller, train.py:304-462) with libdcn's
DeformConv2d on one MI355X.

The network mirrors JittorEDNetDetection (train.py:304-339): conv1 3x3 -> BN -> ReLU, four
DeformConv2d(3, 2, 1) stages 16->32->64->128->256 (128² -> 8²), each + BN + ReLU, global
average pool, a 10-way classifier and a sigmoid box head. The loop mirrors train.py:353-418:
Adam(lr 1e-3, weight decay 1e-4), cross-entropy + 5 x smooth-L1(beta 1) on the box, batch
10. The reference data (prepare_data.py) are MNIST digits pasted on 128² canvases; there
is no network here, so the data are synthetic canvases of the same shape: one of 10
procedurally drawn glyph classes (28x28) at a random position, with its box. The non-DCN
layers are torch; every DeformConv2d runs in libdcn (torch_dcn.DeformConv2d).

    python examples/ednet_train.py [--steps 100] [--impl libdcn|literal]
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "jittor-dcn_amd"))


def glyph(cls: int, rng) -> np.ndarray:
    """28x28 glyph of class cls: strokes whose layout depends on the class."""
    g = np.zeros((28, 28), np.float32)
    k = cls + 1
    for s in range(1 + cls % 3):
        r0 = 4 + (7 * (k + s)) % 18
        g[r0:r0 + 3, 3:25] = 1.0  # horizontal bar
    for s in range(1 + cls // 4):
        c0 = 4 + (5 * (k + 2 * s)) % 18
        g[3:25, c0:c0 + 3] = np.maximum(g[3:25, c0:c0 + 3], 0.8)  # vertical bar
    g += rng.normal(0, 0.05, g.shape).astype(np.float32)
    return np.clip(g, 0, 1)


def make_data(n, seed, size=128):
    """prepare_data.py:create_detection_image's shapes: [n,1,128,128] canvases, a box
    (x1, y1, x2, y2) normalised to the canvas, and a class label."""
    rng = np.random.default_rng(seed)
    imgs = np.zeros((n, 1, size, size), np.float32)
    boxes = np.zeros((n, 4), np.float32)
    labels = rng.integers(0, 10, n)
    for i in range(n):
        x, y = rng.integers(0, size - 28, 2)
        imgs[i, 0, y:y + 28, x:x + 28] = glyph(int(labels[i]), rng)
        boxes[i] = [x / size, y / size, (x + 28) / size, (y + 28) / size]
    return imgs, boxes, labels


class EDNet(nn.Module):
    """train.py:304-339 with a pluggable DeformConv2d class (and activation: the parity
    test swaps ReLU for a smooth one so fp32-vs-f64 comparisons never straddle a ReLU
    mask)."""

    def __init__(self, dcn_cls, num_classes=10, act=F.relu):
        super().__init__()
        self.act = act
        self.conv1 = nn.Conv2d(1, 16, 3, 1, 1)
        self.bn1 = nn.BatchNorm2d(16)
        self.conv2, self.bn2 = dcn_cls(16, 32, 3, 2, 1), nn.BatchNorm2d(32)
        self.conv3, self.bn3 = dcn_cls(32, 64, 3, 2, 1), nn.BatchNorm2d(64)
        self.conv4, self.bn4 = dcn_cls(64, 128, 3, 2, 1), nn.BatchNorm2d(128)
        self.conv5, self.bn5 = dcn_cls(128, 256, 3, 2, 1), nn.BatchNorm2d(256)
        self.fc_cls = nn.Linear(256, num_classes)
        self.fc_bbox = nn.Linear(256, 4)

    def forward(self, x):
        x = self.act(self.bn1(self.conv1(x)))
        for c, bn in ((self.conv2, self.bn2), (self.conv3, self.bn3), (self.conv4, self.bn4),
                      (self.conv5, self.bn5)):
            x = self.act(bn(c(x)))
        x = x.mean(dim=(2, 3))
        return self.fc_cls(x), torch.sigmoid(self.fc_bbox(x))


def smooth_l1(pred, target, beta=1.0):  # train.py:359-363
    d = (pred - target).abs()
    return torch.where(d < beta, 0.5 * d * d / beta, d - 0.5 * beta).mean()


def train(model, imgs, boxes, labels, steps, batch=10, seed=0, log=print):
    p0 = next(model.parameters())
    dev, dt = p0.device, p0.dtype
    opt = torch.optim.Adam(model.parameters(), lr=1e-3, weight_decay=1e-4)  # train.py:351
    rng = np.random.default_rng(seed)
    losses = []
    n = len(imgs)
    order = rng.permutation(n)
    for step in range(steps):
        idx = order[(step * batch) % n:(step * batch) % n + batch]
        if len(idx) < batch:
            order = rng.permutation(n)
            idx = order[:batch]
        xb = torch.from_numpy(imgs[idx]).to(dev, dt)
        yb = torch.from_numpy(labels[idx]).to(dev)
        bb = torch.from_numpy(boxes[idx]).to(dev, dt)
        opt.zero_grad()
        cls, box = model(xb)
        cls_loss = F.cross_entropy(cls, yb)
        box_loss = smooth_l1(box, bb)
        loss = cls_loss + 5.0 * box_loss  # train.py:411
        loss.backward()
        opt.step()
        losses.append(float(loss.item()))
        if log and (step % 20 == 0 or step == steps - 1):
            acc = float((cls.argmax(1) == yb).float().mean())
            log(f"[libdcn] step {step:4d} total {loss.item():.4f} cls {cls_loss.item():.4f} "
                f"bbox {box_loss.item():.4f} acc {acc:.2f}")
    return losses


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--n-train", type=int, default=500)  # prepare_data.py n_train
    args = ap.parse_args()
    import torch_dcn
    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    model = EDNet(torch_dcn.DeformConv2d).to(dev)
    imgs, boxes, labels = make_data(args.n_train, 1)
    t0 = time.perf_counter()
    losses = train(model, imgs, boxes, labels, args.steps)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(f"{args.steps} steps in {el:.2f} s ({el / args.steps * 1e3:.1f} ms/step); "
          f"loss {losses[0]:.4f} -> {np.mean(losses[-10:]):.4f}")


if __name__ == "__main__":
    main()
