// pybind11 module `_tk8s_topo`: CPU-only topology allocator (N2 core). Loaded by the node
// agent's device plugin, which must never initialise the GPU itself.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "tk8s/topology.h"

namespace py = pybind11;

PYBIND11_MODULE(_tk8s_topo, m) {
  m.doc() = "tk8s xGMI-aware GPU set selection (pure C++, no HIP)";
  m.def("link_weight", &tk8s::link_weight, py::arg("type"), py::arg("hops"));
  m.def(
      "preferred_allocation",
      [](int n, const std::vector<int>& weights, const std::vector<int>& available,
         const std::vector<int>& must_include, int size) {
        const auto r = tk8s::preferred_allocation(n, weights, available, must_include, size);
        py::dict d;
        d["devices"] = r.devices;
        d["min_link"] = r.min_link;
        d["total_link"] = r.total_link;
        d["exhaustive"] = r.exhaustive;
        return d;
      },
      py::arg("n"), py::arg("weights"), py::arg("available"), py::arg("must_include"),
      py::arg("size"));
}
