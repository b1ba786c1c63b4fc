// pybind11 entry point of the native host runtime (_host).
#include <pybind11/pybind11.h>
namespace py = pybind11;
namespace slate_host {
void register_runtime(py::module& m);
void register_tile_kernels(py::module& m);
void register_matgen(py::module& m);
void register_eig(py::module& m);
}
PYBIND11_MODULE(_host, m) {
    m.doc() = "slate_amd native host runtime (MOSI table, slab pool, trace, host tile kernels, matgen)";
    slate_host::register_runtime(m);
    slate_host::register_tile_kernels(m);
    slate_host::register_matgen(m);
    slate_host::register_eig(m);
}
