// Host runtime of the framework (C++): asynchronous parameter server, its client, and the
// multi-threaded batch assembler that feeds pinned host buffers for the H2D ingest stream.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace ddl {

class ParamServer {
 public:
  // rule: 0 = add residual (ADAG / DOWNPOUR / EASGD), 1 = DynSGD staleness scaling
  ParamServer(const float* init, int64_t n, int rule, int port);
  ~ParamServer();
  int port() const { return port_; }
  int64_t num_updates();
  void get_center(float* out, int64_t n);
  int64_t size() const { return (int64_t)center_.size(); }
  void stop();

 private:
  void accept_loop();
  void serve(int fd);
  std::vector<float> center_;
  int rule_;
  int port_ = 0;
  int listen_fd_ = -1;
  int64_t num_updates_ = 0;
  std::atomic<bool> running_{false};
  std::mutex mu_, conn_mu_;
  std::thread acceptor_;
  std::vector<std::thread> handlers_;
  std::vector<int> conns_;
};

class PSClient {
 public:
  PSClient(const std::string& host, int port, int worker_id);
  ~PSClient();
  void commit(const float* residual, int64_t n, int64_t last_update);
  int64_t pull(float* out, int64_t n);  // returns the server's num_updates at pull time
  void close();

 private:
  int fd_ = -1;
  int64_t worker_id_;
};

// Assembles mini-batches (optionally shuffled per epoch) from a host array into a ring of
// caller-provided (pinned) buffers with a background thread pool.
class BatchLoader {
 public:
  BatchLoader(const void* x, int64_t rows, int64_t x_row_bytes, const void* y, int64_t y_row_bytes, int64_t batch,
              bool shuffle, uint64_t seed, bool drop_last, int threads);
  ~BatchLoader();
  void set_buffers(const std::vector<uintptr_t>& xbufs, const std::vector<uintptr_t>& ybufs);
  void start_epoch(int64_t epoch);
  int next(int64_t* nrows);  // slot index of the next ready batch, -1 at end of epoch
  void release(int slot);
  int64_t batches_per_epoch() const;

 private:
  void producer();
  void fill(int slot, int64_t b);
  const char* x_;
  const char* y_;
  int64_t rows_, xrb_, yrb_, batch_;
  bool shuffle_, drop_last_;
  uint64_t seed_;
  int threads_;
  std::vector<char*> xb_, yb_;
  std::vector<int64_t> perm_;
  std::vector<int> state_;  // 0 free, 1 filling, 2 ready
  std::vector<int64_t> slot_rows_;
  std::vector<int64_t> slot_batch_;
  int64_t epoch_ = -1, next_fill_ = 0, next_take_ = 0, nbatches_ = 0;
  bool stop_ = false;
  std::mutex mu_;
  std::condition_variable cv_;
  std::thread worker_;
};

}  // namespace ddl
