// Multi-threaded mini-batch assembler (host side of the ingest pipeline).
//
// The reference assembles every mini-batch in Python row by row inside each worker
// (``X = [row[features_col]]``, SURVEY §3.3 hot loop 3).  Here a background thread
// gathers the (optionally per-epoch shuffled) rows of a resident host shard straight
// into a ring of caller-owned pinned buffers, parallelising large gathers over a few
// threads; the Python side overlaps the H2D copy of slot i with compute on slot i-1.
#include <algorithm>
#include <cstring>
#include <numeric>
#include <random>
#include <stdexcept>

#include "ddl_runtime.h"

namespace ddl {

BatchLoader::BatchLoader(const void* x, int64_t rows, int64_t x_row_bytes, const void* y, int64_t y_row_bytes,
                         int64_t batch, bool shuffle, uint64_t seed, bool drop_last, int threads)
    : x_(static_cast<const char*>(x)),
      y_(static_cast<const char*>(y)),
      rows_(rows),
      xrb_(x_row_bytes),
      yrb_(y_row_bytes),
      batch_(batch),
      shuffle_(shuffle),
      drop_last_(drop_last),
      seed_(seed),
      threads_(std::max(1, threads)) {
  if (batch <= 0) throw std::invalid_argument("BatchLoader: batch must be > 0");
  perm_.resize((size_t)rows);
  std::iota(perm_.begin(), perm_.end(), 0);
  worker_ = std::thread([this] { producer(); });
}

BatchLoader::~BatchLoader() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  if (worker_.joinable()) worker_.join();
}

int64_t BatchLoader::batches_per_epoch() const {
  return drop_last_ ? rows_ / batch_ : (rows_ + batch_ - 1) / batch_;
}

void BatchLoader::set_buffers(const std::vector<uintptr_t>& xbufs, const std::vector<uintptr_t>& ybufs) {
  std::lock_guard<std::mutex> g(mu_);
  if (xbufs.empty() || (y_ && ybufs.size() != xbufs.size())) throw std::invalid_argument("BatchLoader: bad buffers");
  xb_.clear();
  yb_.clear();
  for (auto p : xbufs) xb_.push_back(reinterpret_cast<char*>(p));
  for (auto p : ybufs) yb_.push_back(reinterpret_cast<char*>(p));
  state_.assign(xb_.size(), 0);
  slot_rows_.assign(xb_.size(), 0);
  slot_batch_.assign(xb_.size(), -1);
}

void BatchLoader::start_epoch(int64_t epoch) {
  std::unique_lock<std::mutex> l(mu_);
  if (xb_.empty()) throw std::runtime_error("BatchLoader: set_buffers() first");
  // wait until the consumer released every slot of the previous epoch
  cv_.wait(l, [&] { return std::all_of(state_.begin(), state_.end(), [](int s) { return s != 1; }); });
  std::fill(state_.begin(), state_.end(), 0);
  if (shuffle_) {
    std::iota(perm_.begin(), perm_.end(), 0);
    std::mt19937_64 rng(seed_ * 1000003ULL + (uint64_t)epoch);
    std::shuffle(perm_.begin(), perm_.end(), rng);
  }
  epoch_ = epoch;
  nbatches_ = batches_per_epoch();
  next_fill_ = 0;
  next_take_ = 0;
  l.unlock();
  cv_.notify_all();
}

void BatchLoader::fill(int slot, int64_t b) {
  const int64_t r0 = b * batch_;
  const int64_t n = std::min(batch_, rows_ - r0);
  char* xo = xb_[(size_t)slot];
  char* yo = y_ ? yb_[(size_t)slot] : nullptr;
  auto work = [&](int64_t lo, int64_t hi) {
    for (int64_t i = lo; i < hi; ++i) {
      const int64_t src = perm_[(size_t)(r0 + i)];
      std::memcpy(xo + i * xrb_, x_ + src * xrb_, (size_t)xrb_);
      if (yo) std::memcpy(yo + i * yrb_, y_ + src * yrb_, (size_t)yrb_);
    }
  };
  const int64_t bytes = n * (xrb_ + yrb_);
  const int nt = bytes > (8 << 20) ? threads_ : 1;
  if (nt == 1) {
    work(0, n);
  } else {
    std::vector<std::thread> ts;
    for (int t = 0; t < nt; ++t) ts.emplace_back(work, n * t / nt, n * (t + 1) / nt);
    for (auto& t : ts) t.join();
  }
  slot_rows_[(size_t)slot] = n;
}

void BatchLoader::producer() {
  std::unique_lock<std::mutex> l(mu_);
  while (true) {
    cv_.wait(l, [&] {
      if (stop_) return true;
      if (epoch_ < 0 || next_fill_ >= nbatches_ || xb_.empty()) return false;
      return state_[(size_t)(next_fill_ % (int64_t)xb_.size())] == 0;
    });
    if (stop_) return;
    const int slot = (int)(next_fill_ % (int64_t)xb_.size());
    const int64_t b = next_fill_++;
    state_[(size_t)slot] = 1;
    slot_batch_[(size_t)slot] = b;
    l.unlock();
    fill(slot, b);
    l.lock();
    state_[(size_t)slot] = 2;
    cv_.notify_all();
  }
}

int BatchLoader::next(int64_t* nrows) {
  std::unique_lock<std::mutex> l(mu_);
  if (next_take_ >= nbatches_) return -1;
  const int slot = (int)(next_take_ % (int64_t)xb_.size());
  cv_.wait(l, [&] { return stop_ || (state_[(size_t)slot] == 2 && slot_batch_[(size_t)slot] == next_take_); });
  if (stop_) return -1;
  ++next_take_;
  if (nrows) *nrows = slot_rows_[(size_t)slot];
  return slot;
}

void BatchLoader::release(int slot) {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (slot >= 0 && slot < (int)state_.size()) state_[(size_t)slot] = 0;
  }
  cv_.notify_all();
}

}  // namespace ddl
