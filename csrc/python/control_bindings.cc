// pybind11 bindings of the control plane (protocol, server, client, HTTP).
#include <pybind11/pybind11.h>
namespace py = pybind11;
void bind_control_plane(py::module_& m) { (void)m; }
