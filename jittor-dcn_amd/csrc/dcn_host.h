// dcn_host.h — host-side transfer machinery of the host-pointer API (dcn_forward_host,
// dcn_backward_host): the NumPy / Jittor-CPU caller's path (train.py:408-414 through the
// drop-in module). Caller arrays are pageable, so every transfer is staged through a
// handle-owned ring of pinned chunks: the copy into (or out of) chunk i+1 runs on a small
// pool of host threads while the DMA engine moves chunk i, so PCIe and host memory
// bandwidth overlap. r01 copied straight from pageable memory and allocated device
// buffers per call (89 ms/step at config 3).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace dcn {

// Fixed set of worker threads running one parallel memcpy at a time (the caller's thread
// takes a share too). Pieces are 64-B aligned ranges of the copy.
class CopyPool {
 public:
  explicit CopyPool(int nthreads) : n_(std::max(1, nthreads)) {
    for (int i = 1; i < n_; ++i) th_.emplace_back([this, i] { run(i); });
  }
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> lk(m_);
      stop_ = true;
      ++gen_;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  int threads() const { return n_; }
  void copy(void* dst, const void* src, size_t bytes) {
    if (n_ == 1 || bytes < (1u << 20)) {
      std::memcpy(dst, src, bytes);
      return;
    }
    {
      std::lock_guard<std::mutex> lk(m_);
      dst_ = static_cast<char*>(dst);
      src_ = static_cast<const char*>(src);
      bytes_ = bytes;
      pending_.store(n_ - 1);
      ++gen_;
    }
    cv_.notify_all();
    piece(0);
    std::unique_lock<std::mutex> lk(m_);
    done_cv_.wait(lk, [this] { return pending_.load() == 0; });
  }

 private:
  void piece(int i) {
    const size_t per = (bytes_ / n_ + 63) / 64 * 64;
    const size_t lo = std::min(bytes_, per * i), hi = std::min(bytes_, lo + per);
    if (hi > lo) std::memcpy(dst_ + lo, src_ + lo, hi - lo);
  }
  void run(int i) {
    unsigned long seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        if (stop_) return;
      }
      piece(i);
      if (pending_.fetch_sub(1) == 1) {
        std::lock_guard<std::mutex> lk(m_);
        done_cv_.notify_one();
      }
    }
  }
  int n_;
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_, done_cv_;
  unsigned long gen_ = 0;
  bool stop_ = false;
  std::atomic<int> pending_{0};
  char* dst_ = nullptr;
  const char* src_ = nullptr;
  size_t bytes_ = 0;
};

// Pinned staging ring. Transfers are ordered on the stream passed in; h2d returns once
// the last chunk's DMA is enqueued (the source may then be reused by the caller only
// after the stream reaches that point: the host-pointer API synchronises before it
// returns), d2h returns with the data in the destination.
class HostStage {
 public:
  static constexpr int kSlots = 3;
  HostStage(size_t chunk, int threads) : chunk_(chunk), pool_(threads) {}
  ~HostStage() {
    for (int i = 0; i < kSlots; ++i) {
      if (ev_[i]) (void)hipEventDestroy(ev_[i]);
      if (buf_[i]) (void)hipHostFree(buf_[i]);
    }
  }
  hipError_t init() {
    for (int i = 0; i < kSlots; ++i) {
      hipError_t e = hipHostMalloc(&buf_[i], chunk_, hipHostMallocDefault);
      if (e == hipSuccess) e = hipEventCreateWithFlags(&ev_[i], hipEventDisableTiming);
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  }
  int threads() const { return pool_.threads(); }

  hipError_t h2d(void* dst, const void* src, size_t bytes, hipStream_t s) {
    const char* sp = static_cast<const char*>(src);
    char* dp = static_cast<char*>(dst);
    for (size_t off = 0, i = 0; off < bytes; off += chunk_, ++i) {
      const int slot = (int)(i % kSlots);
      const size_t n = std::min(chunk_, bytes - off);
      hipError_t e = wait_slot(slot);  // the slot's previous DMA has read it
      if (e != hipSuccess) return e;
      pool_.copy(buf_[slot], sp + off, n);
      e = hipMemcpyAsync(dp + off, buf_[slot], n, hipMemcpyHostToDevice, s);
      if (e == hipSuccess) e = hipEventRecord(ev_[slot], s);
      if (e != hipSuccess) return e;
      used_[slot] = true;
    }
    return hipSuccess;
  }

  hipError_t d2h(void* dst, const void* src, size_t bytes, hipStream_t s) {
    const char* sp = static_cast<const char*>(src);
    char* dp = static_cast<char*>(dst);
    const size_t nch = (bytes + chunk_ - 1) / chunk_;
    // DMA runs kSlots-1 chunks ahead of the host copies out of the ring
    auto issue = [&](size_t i) -> hipError_t {
      const int slot = (int)(i % kSlots);
      const size_t off = i * chunk_, n = std::min(chunk_, bytes - off);
      hipError_t e = wait_slot(slot);
      if (e == hipSuccess) e = hipMemcpyAsync(buf_[slot], sp + off, n, hipMemcpyDeviceToHost, s);
      if (e == hipSuccess) e = hipEventRecord(ev_[slot], s);
      used_[slot] = true;
      return e;
    };
    for (size_t i = 0; i < std::min(nch, (size_t)kSlots - 1); ++i) {
      hipError_t e = issue(i);
      if (e != hipSuccess) return e;
    }
    for (size_t i = 0; i < nch; ++i) {
      const int slot = (int)(i % kSlots);
      const size_t off = i * chunk_, n = std::min(chunk_, bytes - off);
      if (i + kSlots - 1 < nch) {
        hipError_t e = issue(i + kSlots - 1);
        if (e != hipSuccess) return e;
      }
      hipError_t e = hipEventSynchronize(ev_[slot]);
      if (e != hipSuccess) return e;
      used_[slot] = false;
      pool_.copy(dp + off, buf_[slot], n);
    }
    return hipSuccess;
  }

 private:
  hipError_t wait_slot(int slot) {
    if (!used_[slot]) return hipSuccess;
    used_[slot] = false;
    return hipEventSynchronize(ev_[slot]);
  }
  size_t chunk_;
  CopyPool pool_;
  void* buf_[kSlots] = {nullptr, nullptr, nullptr};
  hipEvent_t ev_[kSlots] = {nullptr, nullptr, nullptr};
  bool used_[kSlots] = {false, false, false};
};

}  // namespace dcn
