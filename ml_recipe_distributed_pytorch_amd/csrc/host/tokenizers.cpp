#include <pybind11/pybind11.h>
namespace py = pybind11;
void hq_register_tokenizers(py::module_& m) {}
