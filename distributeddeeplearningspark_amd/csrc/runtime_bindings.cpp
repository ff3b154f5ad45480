// pybind11 registrations of the host runtime (parameter server, client, batch loader).
// Tensors cross the boundary as contiguous CPU tensors (fp32 for the PS); the GIL is
// released around every blocking network / copy call.
#include <torch/extension.h>

#include "ddl_runtime.h"

namespace py = pybind11;
using namespace ddl;

namespace {

void check_f32_cpu(const at::Tensor& t, const char* what) {
  TORCH_CHECK(!t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous(), what,
              " must be a contiguous fp32 CPU tensor");
}

}  // namespace

void register_trace(py::module& m);  // runtime/trace.cpp

void register_runtime(py::module& m) {
  register_trace(m);
  py::class_<ParamServer>(m, "ParamServer")
      .def(py::init([](const at::Tensor& init, int rule, int port) {
             check_f32_cpu(init, "init");
             return new ParamServer(init.data_ptr<float>(), init.numel(), rule, port);
           }),
           py::arg("init"), py::arg("rule") = 0, py::arg("port") = 0)
      .def_property_readonly("port", &ParamServer::port)
      .def_property_readonly("num_updates", &ParamServer::num_updates)
      .def("get_center",
           [](ParamServer& s, at::Tensor& out) {
             check_f32_cpu(out, "out");
             py::gil_scoped_release r;
             s.get_center(out.data_ptr<float>(), out.numel());
           })
      .def("stop", [](ParamServer& s) {
        py::gil_scoped_release r;
        s.stop();
      });

  py::class_<PSClient>(m, "PSClient")
      .def(py::init([](const std::string& host, int port, int worker_id) {
             py::gil_scoped_release r;
             return new PSClient(host, port, worker_id);
           }),
           py::arg("host"), py::arg("port"), py::arg("worker_id") = 0)
      .def("commit",
           [](PSClient& c, const at::Tensor& residual, int64_t last_update) {
             check_f32_cpu(residual, "residual");
             py::gil_scoped_release r;
             c.commit(residual.data_ptr<float>(), residual.numel(), last_update);
           },
           py::arg("residual"), py::arg("last_update") = 0)
      .def("pull",
           [](PSClient& c, at::Tensor& out) {
             check_f32_cpu(out, "out");
             py::gil_scoped_release r;
             return c.pull(out.data_ptr<float>(), out.numel());
           })
      .def("close", &PSClient::close);

  py::class_<BatchLoader>(m, "BatchLoader")
      .def(py::init([](const at::Tensor& x, c10::optional<at::Tensor> y, int64_t batch, bool shuffle, uint64_t seed,
                       bool drop_last, int threads) {
             TORCH_CHECK(!x.is_cuda() && x.is_contiguous() && x.dim() >= 1, "x must be a contiguous host tensor");
             const int64_t rows = x.size(0);
             const int64_t xrb = rows ? x.nbytes() / rows : 0;
             const void* yp = nullptr;
             int64_t yrb = 0;
             if (y) {
               TORCH_CHECK(!y->is_cuda() && y->is_contiguous() && y->size(0) == rows, "y must match x rows");
               yp = y->data_ptr();
               yrb = rows ? y->nbytes() / rows : 0;
             }
             return new BatchLoader(x.data_ptr(), rows, xrb, yp, yrb, batch, shuffle, seed, drop_last, threads);
           }),
           py::arg("x"), py::arg("y") = py::none(), py::arg("batch") = 32, py::arg("shuffle") = false,
           py::arg("seed") = 0, py::arg("drop_last") = true, py::arg("threads") = 4, py::keep_alive<1, 2>(),
           py::keep_alive<1, 3>())
      .def("set_buffers",
           [](BatchLoader& l, const std::vector<at::Tensor>& xs, const std::vector<at::Tensor>& ys) {
             std::vector<uintptr_t> xp, yp;
             for (auto& t : xs) xp.push_back(reinterpret_cast<uintptr_t>(t.data_ptr()));
             for (auto& t : ys) yp.push_back(reinterpret_cast<uintptr_t>(t.data_ptr()));
             l.set_buffers(xp, yp);
           })
      .def("start_epoch",
           [](BatchLoader& l, int64_t e) {
             py::gil_scoped_release r;
             l.start_epoch(e);
           })
      .def("next",
           [](BatchLoader& l) {
             int64_t n = 0;
             int s;
             {
               py::gil_scoped_release r;
               s = l.next(&n);
             }
             return py::make_tuple(s, n);
           })
      .def("release", &BatchLoader::release)
      .def_property_readonly("batches_per_epoch", &BatchLoader::batches_per_epoch);
}
