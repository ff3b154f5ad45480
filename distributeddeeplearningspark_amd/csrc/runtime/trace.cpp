// Host tracing runtime: roctx ranges (visible in `rocprofv3 --marker-trace` next to the
// kernel trace) and a lock-free-ish in-process span recorder that the Python tracer dumps
// as a Chrome/Perfetto JSON trace (utils/tracing.py).
#include <chrono>
#include <mutex>
#include <string>
#include <vector>

#include <rocprofiler-sdk-roctx/roctx.h>
#include <torch/extension.h>

namespace py = pybind11;

namespace {

struct Span {
  std::string name;
  int64_t t0_ns, t1_ns;
  int depth;
};

std::mutex g_mu;
std::vector<Span> g_spans;
std::vector<std::pair<std::string, int64_t>> g_open;
bool g_record = false;

int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

void push(const std::string& name) {
  roctxRangePushA(name.c_str());
  if (g_record) {
    std::lock_guard<std::mutex> g(g_mu);
    g_open.emplace_back(name, now_ns());
  }
}

void pop() {
  roctxRangePop();
  if (g_record) {
    std::lock_guard<std::mutex> g(g_mu);
    if (!g_open.empty()) {
      auto o = g_open.back();
      g_open.pop_back();
      g_spans.push_back({o.first, o.second, now_ns(), (int)g_open.size()});
    }
  }
}

}  // namespace

void register_trace(py::module& m) {
  m.def("trace_push", &push, "roctx range push (+ host span when recording)");
  m.def("trace_pop", &pop, "roctx range pop");
  m.def("trace_mark", [](const std::string& s) { roctxMarkA(s.c_str()); });
  m.def("trace_record", [](bool on) {
    std::lock_guard<std::mutex> g(g_mu);
    g_record = on;
  });
  m.def("trace_now_ns", &now_ns);
  m.def("trace_collect", []() {
    std::lock_guard<std::mutex> g(g_mu);
    py::list out;
    for (auto& s : g_spans) out.append(py::make_tuple(s.name, s.t0_ns, s.t1_ns, s.depth));
    g_spans.clear();
    return out;
  });
}
