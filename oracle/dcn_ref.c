/*
 * dcn_ref.c — fp32 C/OpenMP restatement of the DeformConv2d hot path.
 * TEST INFRASTRUCTURE ONLY: the checker for tests/ and __graft_entry__.smoke(),
 * and the timed CPU baseline ("kind": "port") in bench.py. Never linked into
 * or called by the product library (jittor-dcn_amd/).
 *
 * Restates /root/reference/deform_conv.py:56-81 plus its Jittor autodiff in
 * plain fp32 loops (the reference is a fp32 CPU module, train.py:301):
 *   offset conv            deform_conv.py:16-21, :58
 *   offset layout Δx|Δy    deform_conv.py:62
 *   base grid (w, h)       deform_conv.py:64-68 (no tap offsets, no stride)
 *   normalise by out size  deform_conv.py:34-39, grid = [norm_y, norm_x]
 *   bilinear, zeros, align_corners=True   deform_conv.py:47-52
 *   k = n*C + c columns vs weight.reshape(O,-1)   deform_conv.py:72-76
 *   bias                   deform_conv.py:79-80
 * Must be compiled WITHOUT -ffast-math and with -ffp-contract=off: the
 * coordinate chain rounds like the reference's fp32 op sequence.
 * Extensions dil/G as in oracle/dcn_oracle.py (no reference oracle).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef struct {
  int B, C, H, W, O, kh, kw, sh, sw, ph, pw, dh, dw, G, has_bias;
} dcnref_desc;

typedef struct {
  int Ho, Wo, N, K, HW, HWi, Cg, J;
} geo_t;

static int geo(const dcnref_desc* d, geo_t* g) {
  g->Ho = (d->H + 2 * d->ph - d->dh * (d->kh - 1) - 1) / d->sh + 1;
  g->Wo = (d->W + 2 * d->pw - d->dw * (d->kw - 1) - 1) / d->sw + 1;
  if (g->Ho < 2 || g->Wo < 2 || d->C % d->G) return -1;
  g->N = d->kh * d->kw;
  g->K = g->N * d->C;
  g->HW = g->Ho * g->Wo;
  g->HWi = d->H * d->W;
  g->Cg = d->C / d->G;
  g->J = 2 * g->N * d->G;
  return 0;
}

int dcnref_out_shape(const dcnref_desc* d, int* Ho, int* Wo) {
  geo_t g;
  if (geo(d, &g)) return -1;
  *Ho = g.Ho;
  *Wo = g.Wo;
  return 0;
}

int dcnref_num_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

void dcnref_set_threads(int n) {
#ifdef _OPENMP
  if (n > 0) omp_set_num_threads(n);
#else
  (void)n;
#endif
}

/* sampling coordinates, fp32, reference op order */
static void coord(int h, int w, float dx, float dy, const dcnref_desc* d, const geo_t* g,
                  float* iy, float* ix) {
  float cx = (float)w + dx;
  float nx = cx / (float)(g->Wo - 1);
  nx = nx * 2.0f;
  nx = nx - 1.0f;
  *iy = ((nx + 1.0f) / 2.0f) * (float)(d->H - 1);
  float cy = (float)h + dy;
  float ny = cy / (float)(g->Ho - 1);
  ny = ny * 2.0f;
  ny = ny - 1.0f;
  *ix = ((ny + 1.0f) / 2.0f) * (float)(d->W - 1);
}

typedef struct {
  int r0, c0, ok;
  float fr, fc;
} tap_t;

static tap_t mk_tap(float iy, float ix, const dcnref_desc* d) {
  tap_t t;
  float r0f = floorf(iy), c0f = floorf(ix);
  t.ok = (r0f >= -1.0f) && (r0f <= (float)(d->H - 1)) && (c0f >= -1.0f) && (c0f <= (float)(d->W - 1));
  t.r0 = t.ok ? (int)r0f : 0;
  t.c0 = t.ok ? (int)c0f : 0;
  t.fr = t.ok ? iy - r0f : 0.f;
  t.fc = t.ok ? ix - c0f : 0.f;
  return t;
}

static float px(const float* xp, int r, int c, const dcnref_desc* d) {
  return (r >= 0 && r < d->H && c >= 0 && c < d->W) ? xp[r * d->W + c] : 0.f;
}

static tap_t tap_of(const dcnref_desc* d, const geo_t* g, const float* offb, int gi, int n, int m) {
  const float* ob = offb + (size_t)gi * 2 * g->N * g->HW;
  int h = m / g->Wo, w = m % g->Wo;
  float iy, ix;
  coord(h, w, ob[(size_t)n * g->HW + m], ob[(size_t)(g->N + n) * g->HW + m], d, g, &iy, &ix);
  return mk_tap(iy, ix, d);
}

/* ---- offset conv (one image) ---- */
static void offconv_fwd_img(const dcnref_desc* d, const geo_t* g, const float* xb, const float* wo,
                            const float* bo, float* offb) {
  int KK = d->kh * d->kw;
#pragma omp parallel for schedule(static)
  for (int j = 0; j < g->J; ++j) {
    float* o = offb + (size_t)j * g->HW;
    for (int m = 0; m < g->HW; ++m) o[m] = 0.f;
    for (int c = 0; c < d->C; ++c)
      for (int i = 0; i < d->kh; ++i)
        for (int k = 0; k < d->kw; ++k) {
          float wv = wo[((size_t)j * d->C + c) * KK + i * d->kw + k];
          const float* xc = xb + (size_t)c * g->HWi;
          for (int ho = 0; ho < g->Ho; ++ho) {
            int y = ho * d->sh - d->ph + i * d->dh;
            if (y < 0 || y >= d->H) continue;
            for (int wo_ = 0; wo_ < g->Wo; ++wo_) {
              int xx = wo_ * d->sw - d->pw + k * d->dw;
              if (xx < 0 || xx >= d->W) continue;
              o[ho * g->Wo + wo_] += wv * xc[y * d->W + xx];
            }
          }
        }
    for (int m = 0; m < g->HW; ++m) o[m] += bo[j];
  }
}

/* col[k = n*C + c][m] for one image */
static void im2col_img(const dcnref_desc* d, const geo_t* g, const float* xb, const float* offb,
                       float* col) {
#pragma omp parallel for schedule(static)
  for (int k = 0; k < g->K; ++k) {
    int n = k / d->C, c = k % d->C, gi = c / g->Cg;
    const float* xp = xb + (size_t)c * g->HWi;
    float* dst = col + (size_t)k * g->HW;
    for (int m = 0; m < g->HW; ++m) {
      tap_t t = tap_of(d, g, offb, gi, n, m);
      float v = 0.f;
      if (t.ok) {
        float gr = 1.0f - t.fr, gc = 1.0f - t.fc;
        v = (gr * gc) * px(xp, t.r0, t.c0, d);
        v = fmaf(gr * t.fc, px(xp, t.r0, t.c0 + 1, d), v);
        v = fmaf(t.fr * gc, px(xp, t.r0 + 1, t.c0, d), v);
        v = fmaf(t.fr * t.fc, px(xp, t.r0 + 1, t.c0 + 1, d), v);
      }
      dst[m] = v;
    }
  }
}

int dcnref_forward(const dcnref_desc* d, const float* x, const float* w_off, const float* b_off,
                   const float* w, const float* b, float* out, float* off) {
  geo_t g;
  if (geo(d, &g)) return -1;
  float* col = (float*)malloc((size_t)g.K * g.HW * sizeof(float));
  if (!col) return -2;
  for (int bi = 0; bi < d->B; ++bi) {
    const float* xb = x + (size_t)bi * d->C * g.HWi;
    float* offb = off + (size_t)bi * g.J * g.HW;
    offconv_fwd_img(d, &g, xb, w_off, b_off, offb);
    im2col_img(d, &g, xb, offb, col);
    float* ob = out + (size_t)bi * d->O * g.HW;
#pragma omp parallel for schedule(static)
    for (int o = 0; o < d->O; ++o) {
      float* dst = ob + (size_t)o * g.HW;
      for (int m = 0; m < g.HW; ++m) dst[m] = 0.f;
      const float* wr = w + (size_t)o * g.K; /* W read as [O][n*C+c] (Q5) */
      for (int k = 0; k < g.K; ++k) {
        float wv = wr[k];
        const float* cr = col + (size_t)k * g.HW;
        for (int m = 0; m < g.HW; ++m) dst[m] = fmaf(wv, cr[m], dst[m]);
      }
      if (d->has_bias)
        for (int m = 0; m < g.HW; ++m) dst[m] += b[o];
    }
  }
  free(col);
  return 0;
}

/* deform_conv.py:59-80 only: the sampling + GEMM + bias from GIVEN offsets (the device's),
 * so a test can compare a device forward without the knife edges of a re-derived offset
 * (used for the bf16 path, whose offsets are rounded to bf16 before sampling). */
int dcnref_forward_from_offsets(const dcnref_desc* d, const float* x, const float* off,
                                const float* w, const float* b, float* out) {
  geo_t g;
  if (geo(d, &g)) return -1;
  float* col = (float*)malloc((size_t)g.K * g.HW * sizeof(float));
  if (!col) return -2;
  for (int bi = 0; bi < d->B; ++bi) {
    const float* xb = x + (size_t)bi * d->C * g.HWi;
    im2col_img(d, &g, xb, off + (size_t)bi * g.J * g.HW, col);
    float* ob = out + (size_t)bi * d->O * g.HW;
#pragma omp parallel for schedule(static)
    for (int o = 0; o < d->O; ++o) {
      float* dst = ob + (size_t)o * g.HW;
      for (int m = 0; m < g.HW; ++m) dst[m] = 0.f;
      const float* wr = w + (size_t)o * g.K;
      for (int k = 0; k < g.K; ++k) {
        float wv = wr[k];
        const float* cr = col + (size_t)k * g.HW;
        for (int m = 0; m < g.HW; ++m) dst[m] = fmaf(wv, cr[m], dst[m]);
      }
      if (d->has_bias)
        for (int m = 0; m < g.HW; ++m) dst[m] += b[o];
    }
  }
  free(col);
  return 0;
}

int dcnref_backward(const dcnref_desc* d, const float* x, const float* off, const float* w_off,
                    const float* w, const float* gout, float* gx, float* gw, float* gb,
                    float* gw_off, float* gb_off, float* goff_out) {
  geo_t g;
  if (geo(d, &g)) return -1;
  const int KK = d->kh * d->kw;
  float* col = (float*)malloc((size_t)g.K * g.HW * sizeof(float));
  float* dcol = (float*)malloc((size_t)g.K * g.HW * sizeof(float));
  float* goff = (float*)malloc((size_t)g.J * g.HW * sizeof(float));
  /* the four parameter reductions (sums over B*Ho*Wo pixels) accumulate in double, so the
   * checker's own rounding stays far below the 1e-4 reduction tolerance at full size */
  const size_t nwo = (size_t)g.J * d->C * KK;
  double* aw = (double*)calloc((size_t)d->O * g.K, sizeof(double));
  double* ab = (double*)calloc((size_t)d->O, sizeof(double));
  double* awo = (double*)calloc(nwo, sizeof(double));
  double* abo = (double*)calloc((size_t)g.J, sizeof(double));
  if (!col || !dcol || !goff || !aw || !ab || !awo || !abo) {
    free(col);
    free(dcol);
    free(goff);
    free(aw);
    free(ab);
    free(awo);
    free(abo);
    return -2;
  }
  memset(gx, 0, (size_t)d->B * d->C * g.HWi * sizeof(float));
  for (int bi = 0; bi < d->B; ++bi) {
    const float* xb = x + (size_t)bi * d->C * g.HWi;
    const float* offb = off + (size_t)bi * g.J * g.HW;
    const float* gob = gout + (size_t)bi * d->O * g.HW;
    float* gxb = gx + (size_t)bi * d->C * g.HWi;
    im2col_img(d, &g, xb, offb, col);
    if (d->has_bias)
      for (int o = 0; o < d->O; ++o) {
        double s = 0.0;
        for (int m = 0; m < g.HW; ++m) s += gob[(size_t)o * g.HW + m];
        ab[o] += s;
      }
      /* ∂W[o][k] += Σ_m ∂out[o][m] col[k][m] */
#pragma omp parallel for schedule(static)
    for (int o = 0; o < d->O; ++o)
      for (int k = 0; k < g.K; ++k) {
        const float* a = gob + (size_t)o * g.HW;
        const float* c = col + (size_t)k * g.HW;
        double s = 0.0;
        for (int m = 0; m < g.HW; ++m) s += (double)a[m] * c[m];
        aw[(size_t)o * g.K + k] += s;
      }
      /* ∂col[k][m] = Σ_o W[o][k] ∂out[o][m] */
#pragma omp parallel for schedule(static)
    for (int k = 0; k < g.K; ++k) {
      float* dst = dcol + (size_t)k * g.HW;
      for (int m = 0; m < g.HW; ++m) dst[m] = 0.f;
      for (int o = 0; o < d->O; ++o) {
        float wv = w[(size_t)o * g.K + k];
        const float* a = gob + (size_t)o * g.HW;
        for (int m = 0; m < g.HW; ++m) dst[m] = fmaf(wv, a[m], dst[m]);
      }
    }
    /* sampling backward: ∂off (reduce over channels of the group), ∂x scatter */
    const float sy = (float)(d->H - 1) / (float)(g.Wo - 1);
    const float sx = (float)(d->W - 1) / (float)(g.Ho - 1);
#pragma omp parallel for schedule(static)
    for (int t = 0; t < d->G * g.N; ++t) {
      int gi = t / g.N, n = t % g.N;
      for (int m = 0; m < g.HW; ++m) {
        tap_t tp = tap_of(d, &g, offb, gi, n, m);
        float diy = 0.f, dix = 0.f;
        if (tp.ok) {
          float gr = 1.0f - tp.fr, gc = 1.0f - tp.fc;
          for (int cl = 0; cl < g.Cg; ++cl) {
            int c = gi * g.Cg + cl;
            float gv = dcol[((size_t)n * d->C + c) * g.HW + m];
            const float* xp = xb + (size_t)c * g.HWi;
            float x00 = px(xp, tp.r0, tp.c0, d), x01 = px(xp, tp.r0, tp.c0 + 1, d);
            float x10 = px(xp, tp.r0 + 1, tp.c0, d), x11 = px(xp, tp.r0 + 1, tp.c0 + 1, d);
            diy = fmaf(gv, fmaf(tp.fc, x11 - x01, gc * (x10 - x00)), diy);
            dix = fmaf(gv, fmaf(tp.fr, x11 - x10, gr * (x01 - x00)), dix);
          }
        }
        goff[((size_t)gi * 2 * g.N + n) * g.HW + m] = diy * sy;
        goff[((size_t)gi * 2 * g.N + g.N + n) * g.HW + m] = dix * sx;
      }
    }
    /* ∂x scatter, parallel over channels (each thread owns a channel plane) */
#pragma omp parallel for schedule(static)
    for (int c = 0; c < d->C; ++c) {
      int gi = c / g.Cg;
      float* gxp = gxb + (size_t)c * g.HWi;
      for (int n = 0; n < g.N; ++n)
        for (int m = 0; m < g.HW; ++m) {
          tap_t tp = tap_of(d, &g, offb, gi, n, m);
          if (!tp.ok) continue;
          float gv = dcol[((size_t)n * d->C + c) * g.HW + m];
          float gr = 1.0f - tp.fr, gc = 1.0f - tp.fc;
          int r0 = tp.r0, c0 = tp.c0;
          float wts[4] = {gr * gc, gr * tp.fc, tp.fr * gc, tp.fr * tp.fc};
          int rr[4] = {r0, r0, r0 + 1, r0 + 1}, cc[4] = {c0, c0 + 1, c0, c0 + 1};
          for (int q = 0; q < 4; ++q)
            if (rr[q] >= 0 && rr[q] < d->H && cc[q] >= 0 && cc[q] < d->W)
              gxp[rr[q] * d->W + cc[q]] += gv * wts[q];
        }
    }
    /* offset conv backward */
#pragma omp parallel for schedule(static)
    for (int j = 0; j < g.J; ++j) {
      const float* gj = goff + (size_t)j * g.HW;
      double s = 0.0;
      for (int m = 0; m < g.HW; ++m) s += gj[m];
      abo[j] += s;
      for (int c = 0; c < d->C; ++c)
        for (int i = 0; i < d->kh; ++i)
          for (int k = 0; k < d->kw; ++k) {
            const float* xc = xb + (size_t)c * g.HWi;
            double acc = 0.0;
            for (int ho = 0; ho < g.Ho; ++ho) {
              int y = ho * d->sh - d->ph + i * d->dh;
              if (y < 0 || y >= d->H) continue;
              for (int wo_ = 0; wo_ < g.Wo; ++wo_) {
                int xx = wo_ * d->sw - d->pw + k * d->dw;
                if (xx < 0 || xx >= d->W) continue;
                acc += (double)gj[ho * g.Wo + wo_] * xc[y * d->W + xx];
              }
            }
            awo[((size_t)j * d->C + c) * KK + i * d->kw + k] += acc;
          }
    }
#pragma omp parallel for schedule(static)
    for (int c = 0; c < d->C; ++c) {
      float* gxp = gxb + (size_t)c * g.HWi;
      for (int j = 0; j < g.J; ++j)
        for (int i = 0; i < d->kh; ++i)
          for (int k = 0; k < d->kw; ++k) {
            float wv = w_off[((size_t)j * d->C + c) * KK + i * d->kw + k];
            const float* gj = goff + (size_t)j * g.HW;
            for (int ho = 0; ho < g.Ho; ++ho) {
              int y = ho * d->sh - d->ph + i * d->dh;
              if (y < 0 || y >= d->H) continue;
              for (int wo_ = 0; wo_ < g.Wo; ++wo_) {
                int xx = wo_ * d->sw - d->pw + k * d->dw;
                if (xx < 0 || xx >= d->W) continue;
                gxp[y * d->W + xx] += wv * gj[ho * g.Wo + wo_];
              }
            }
          }
    }
    if (goff_out) memcpy(goff_out + (size_t)bi * g.J * g.HW, goff, (size_t)g.J * g.HW * sizeof(float));
  }
  for (size_t i = 0; i < (size_t)d->O * g.K; ++i) gw[i] = (float)aw[i];
  if (d->has_bias)
    for (int o = 0; o < d->O; ++o) gb[o] = (float)ab[o];
  for (size_t i = 0; i < nwo; ++i) gw_off[i] = (float)awo[i];
  for (int j = 0; j < g.J; ++j) gb_off[j] = (float)abo[j];
  free(col);
  free(dcol);
  free(goff);
  free(aw);
  free(ab);
  free(awo);
  free(abo);
  return 0;
}
