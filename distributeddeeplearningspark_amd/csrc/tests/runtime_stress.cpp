// Host-runtime stress test, built with -fsanitize=address,undefined and -fsanitize=thread by
// tests/test_sanitizers.py (GPU sanitizers are not available on the MI355X pool; the native
// runtime that is concurrent — the parameter server and the batch loader — is host code).
//
//  * ParamServer: W worker threads (own PSClient each) commit C residuals of ones and pull,
//    concurrently; the ADD rule must end at init + W*C with W*C updates, DynSGD must see every
//    commit (num_updates) with bounded scaling.
//  * BatchLoader: E shuffled epochs over R rows into a ring of S buffers, consumer on the main
//    thread; every epoch must deliver each row exactly once with x / y rows kept together.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <set>
#include <thread>
#include <vector>

#include "ddl_runtime.h"

using namespace ddl;

#define CHECK(cond, ...)                                \
  do {                                                  \
    if (!(cond)) {                                      \
      std::fprintf(stderr, "FAILED %s: ", #cond);       \
      std::fprintf(stderr, __VA_ARGS__);                \
      std::fprintf(stderr, "\n");                       \
      return 1;                                         \
    }                                                   \
  } while (0)

static int test_param_server(int rule) {
  const int64_t n = 1000;
  const int W = 6, Cm = 40;
  std::vector<float> init(n);
  for (int64_t i = 0; i < n; ++i) init[i] = (float)i;
  ParamServer ps(init.data(), n, rule, 0);
  std::vector<std::thread> ts;
  std::vector<int> ok(W, 0);
  for (int w = 0; w < W; ++w)
    ts.emplace_back([&, w] {
      PSClient c("127.0.0.1", ps.port(), w);
      std::vector<float> buf(n), ones(n, 1.f);
      int64_t last = c.pull(buf.data(), n);
      for (int i = 0; i < Cm; ++i) {
        c.commit(ones.data(), n, last);
        last = c.pull(buf.data(), n);
      }
      c.close();
      ok[w] = 1;
    });
  for (auto& t : ts) t.join();
  for (int w = 0; w < W; ++w) CHECK(ok[w], "worker %d", w);
  CHECK(ps.num_updates() == (int64_t)W * Cm, "num_updates %lld", (long long)ps.num_updates());
  std::vector<float> c(n);
  ps.get_center(c.data(), n);
  for (int64_t i = 0; i < n; ++i) {
    const float d = c[i] - init[i];
    if (rule == 0) CHECK(std::fabs(d - W * Cm) < 1e-3f, "ADD center[%lld] delta %f", (long long)i, d);
    else CHECK(d > 0.f && d <= W * Cm + 1e-3f, "DynSGD center[%lld] delta %f", (long long)i, d);
  }
  ps.stop();
  return 0;
}

static int test_loader() {
  const int64_t R = 1003, B = 32, XR = 64;
  std::vector<float> x((size_t)(R * XR));
  std::vector<int64_t> y((size_t)R);
  for (int64_t r = 0; r < R; ++r) {
    y[(size_t)r] = r;
    for (int64_t k = 0; k < XR; ++k) x[(size_t)(r * XR + k)] = (float)(r * 1000 + k);
  }
  const int S = 3;
  std::vector<std::vector<float>> xb(S, std::vector<float>((size_t)(B * XR)));
  std::vector<std::vector<int64_t>> yb(S, std::vector<int64_t>((size_t)B));
  BatchLoader L(x.data(), R, XR * 4, y.data(), 8, B, true, 7, false, 4);
  std::vector<uintptr_t> xp, yp;
  for (int s = 0; s < S; ++s) {
    xp.push_back(reinterpret_cast<uintptr_t>(xb[s].data()));
    yp.push_back(reinterpret_cast<uintptr_t>(yb[s].data()));
  }
  L.set_buffers(xp, yp);
  for (int e = 0; e < 4; ++e) {
    L.start_epoch(e);
    std::set<int64_t> seen;
    int64_t nrows = 0;
    for (int slot; (slot = L.next(&nrows)) >= 0;) {
      for (int64_t i = 0; i < nrows; ++i) {
        const int64_t r = yb[slot][(size_t)i];
        CHECK(r >= 0 && r < R, "row id %lld", (long long)r);
        CHECK(xb[slot][(size_t)(i * XR + 5)] == (float)(r * 1000 + 5), "x/y rows out of step");
        CHECK(seen.insert(r).second, "row %lld twice in epoch %d", (long long)r, e);
      }
      L.release(slot);
    }
    CHECK((int64_t)seen.size() == R, "epoch %d delivered %zu rows", e, seen.size());
  }
  return 0;
}

int main() {
  if (test_param_server(0)) return 1;
  if (test_param_server(1)) return 1;
  if (test_loader()) return 1;
  std::printf("runtime stress: ok\n");
  return 0;
}
