// Native asynchronous parameter server + client (TCP), the exact dist-keras protocol
// behind the reference's ADAG / DynSGD / DOWNPOUR trainers:
//   * the driver hosts the center variable (fp32) and an update counter;
//   * each worker connection is served by its own thread; one mutex guards the center;
//   * 'c' commit: center += scale * residual  (ADAG/DOWNPOUR/EASGD: scale 1;
//                 DynSGD: scale 1/(num_updates - last_update + 1), the staleness rule);
//     num_updates += 1
//   * 'p' pull  : returns (num_updates, center)
//   * 's' stop  : closes the connection.
// Framing: 1-byte action, fixed-width little-endian headers, raw fp32 payload (no pickle).
// The synchronous RCCL path (trainers' default) is faster on MI355X; this server exists
// for semantic parity (true asynchrony, stale updates) and for CPU executors.
#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "ddl_runtime.h"

namespace ddl {

namespace {

bool send_all(int fd, const void* buf, size_t n) {
  const char* p = static_cast<const char*>(buf);
  while (n) {
    ssize_t k = ::send(fd, p, n, MSG_NOSIGNAL);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return false;
    p += k;
    n -= (size_t)k;
  }
  return true;
}

bool recv_all(int fd, void* buf, size_t n) {
  char* p = static_cast<char*>(buf);
  while (n) {
    ssize_t k = ::recv(fd, p, n, 0);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return false;
    p += k;
    n -= (size_t)k;
  }
  return true;
}

void set_nodelay(int fd) {
  int one = 1;
  ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
}

}  // namespace

ParamServer::ParamServer(const float* init, int64_t n, int rule, int port)
    : center_(init, init + n), rule_(rule) {
  listen_fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
  if (listen_fd_ < 0) throw std::runtime_error("ParamServer: socket() failed");
  int one = 1;
  ::setsockopt(listen_fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in addr{};
  addr.sin_family = AF_INET;
  addr.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  addr.sin_port = htons((uint16_t)port);
  if (::bind(listen_fd_, (sockaddr*)&addr, sizeof(addr)) != 0) {
    ::close(listen_fd_);
    throw std::runtime_error("ParamServer: bind failed on port " + std::to_string(port));
  }
  socklen_t len = sizeof(addr);
  ::getsockname(listen_fd_, (sockaddr*)&addr, &len);
  port_ = ntohs(addr.sin_port);
  if (::listen(listen_fd_, 128) != 0) throw std::runtime_error("ParamServer: listen failed");
  running_ = true;
  acceptor_ = std::thread([this] { accept_loop(); });
}

ParamServer::~ParamServer() { stop(); }

void ParamServer::accept_loop() {
  while (running_) {
    int fd = ::accept(listen_fd_, nullptr, nullptr);
    if (fd < 0) {
      if (!running_) break;
      if (errno == EINTR) continue;
      break;
    }
    set_nodelay(fd);
    std::lock_guard<std::mutex> g(conn_mu_);
    conns_.push_back(fd);
    handlers_.emplace_back([this, fd] { serve(fd); });
  }
}

void ParamServer::serve(int fd) {
  std::vector<float> buf;
  while (running_) {
    char action;
    if (!recv_all(fd, &action, 1)) break;
    if (action == 'c') {
      int64_t hdr[3];  // worker_id, last_update, n
      if (!recv_all(fd, hdr, sizeof(hdr))) break;
      const int64_t n = hdr[2];
      if (n != (int64_t)center_.size()) break;
      buf.resize((size_t)n);
      if (!recv_all(fd, buf.data(), sizeof(float) * (size_t)n)) break;
      std::lock_guard<std::mutex> g(mu_);
      float scale = 1.f;
      if (rule_ == 1) scale = 1.f / (float)(num_updates_ - hdr[1] + 1);  // DynSGD staleness
      float* c = center_.data();
      for (int64_t i = 0; i < n; ++i) c[i] += scale * buf[(size_t)i];
      ++num_updates_;
    } else if (action == 'p') {
      std::vector<float> snap;
      int64_t hdr[2];
      {
        std::lock_guard<std::mutex> g(mu_);
        snap = center_;
        hdr[0] = num_updates_;
      }
      hdr[1] = (int64_t)snap.size();
      if (!send_all(fd, hdr, sizeof(hdr)) || !send_all(fd, snap.data(), sizeof(float) * snap.size())) break;
    } else {
      break;  // 's' or unknown: close
    }
  }
  ::close(fd);
}

int64_t ParamServer::num_updates() {
  std::lock_guard<std::mutex> g(mu_);
  return num_updates_;
}

void ParamServer::get_center(float* out, int64_t n) {
  std::lock_guard<std::mutex> g(mu_);
  if (n != (int64_t)center_.size()) throw std::runtime_error("ParamServer::get_center: size mismatch");
  std::memcpy(out, center_.data(), sizeof(float) * (size_t)n);
}

void ParamServer::stop() {
  if (!running_.exchange(false)) return;
  ::shutdown(listen_fd_, SHUT_RDWR);
  ::close(listen_fd_);
  if (acceptor_.joinable()) acceptor_.join();
  {
    std::lock_guard<std::mutex> g(conn_mu_);
    for (int fd : conns_) ::shutdown(fd, SHUT_RDWR);
  }
  for (auto& t : handlers_)
    if (t.joinable()) t.join();
  handlers_.clear();
}

// ------------------------------------------------------------------------------ client
PSClient::PSClient(const std::string& host, int port, int worker_id) : worker_id_(worker_id) {
  fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
  if (fd_ < 0) throw std::runtime_error("PSClient: socket() failed");
  sockaddr_in addr{};
  addr.sin_family = AF_INET;
  addr.sin_port = htons((uint16_t)port);
  if (::inet_pton(AF_INET, host.c_str(), &addr.sin_addr) != 1) throw std::runtime_error("PSClient: bad host " + host);
  int tries = 0;
  while (::connect(fd_, (sockaddr*)&addr, sizeof(addr)) != 0) {
    if (++tries > 200) throw std::runtime_error("PSClient: cannot connect to parameter server");
    ::usleep(50000);
  }
  set_nodelay(fd_);
}

PSClient::~PSClient() { close(); }

void PSClient::commit(const float* residual, int64_t n, int64_t last_update) {
  const char a = 'c';
  const int64_t hdr[3] = {worker_id_, last_update, n};
  if (!send_all(fd_, &a, 1) || !send_all(fd_, hdr, sizeof(hdr)) || !send_all(fd_, residual, sizeof(float) * (size_t)n))
    throw std::runtime_error("PSClient: commit failed");
}

int64_t PSClient::pull(float* out, int64_t n) {
  const char a = 'p';
  if (!send_all(fd_, &a, 1)) throw std::runtime_error("PSClient: pull failed");
  int64_t hdr[2];
  if (!recv_all(fd_, hdr, sizeof(hdr))) throw std::runtime_error("PSClient: pull header failed");
  if (hdr[1] != n) throw std::runtime_error("PSClient: center size mismatch");
  if (!recv_all(fd_, out, sizeof(float) * (size_t)n)) throw std::runtime_error("PSClient: pull payload failed");
  return hdr[0];
}

void PSClient::close() {
  if (fd_ >= 0) {
    const char a = 's';
    send_all(fd_, &a, 1);
    ::close(fd_);
    fd_ = -1;
  }
}

}  // namespace ddl
