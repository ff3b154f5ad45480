// pybind11 registrations of the host runtime (parameter server, ingest pipeline).
#include <torch/extension.h>
namespace py = pybind11;

void register_runtime(py::module& m) { (void)m; }
