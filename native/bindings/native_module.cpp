// pybind11 module `_tk8s_native`: HIP kernels, node probes and the RCCL validator for gfx950.
//
// Two levels of API:
//  * probes (*_probe, gpuinfo_json, rccl_allreduce): self-contained, allocate their own
//    buffers, return a JSON string — what the node agent / validation pods use.
//  * raw launchers (hbm_fill, philox_fill, md5_tree, ar_fill, ar_check, stream_copy): take
//    device pointers and a hipStream_t as integers (e.g. torch tensor.data_ptr() and
//    torch.cuda.current_stream().cuda_stream) — what the numerics tests use.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "tk8s/kernels.h"
#include "tk8s/probes.h"
#include "tk8s/rccl_bench.h"

namespace py = pybind11;
using tk8s::DType;
using tk8s::StoreMode;

namespace {

template <class T> T* ptr(uintptr_t p) { return reinterpret_cast<T*>(p); }
hipStream_t stream_of(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

StoreMode mode_of(const std::string& m) {
  if (m == "nontemporal" || m == "nt") return StoreMode::kNonTemporal;
  if (m == "plain") return StoreMode::kPlain;
  throw std::invalid_argument("mode must be 'nontemporal' or 'plain'");
}

DType dtype_of(const std::string& d) {
  if (d == "float32" || d == "f32" || d == "fp32") return DType::kF32;
  if (d == "bfloat16" || d == "bf16") return DType::kBF16;
  throw std::invalid_argument("dtype must be 'float32' or 'bfloat16'");
}

}  // namespace

PYBIND11_MODULE(_tk8s_native, m) {
  m.doc() = "tk8s gfx950 validation kernels (HIP) and RCCL all-reduce validator";
  using G = py::call_guard<py::gil_scoped_release>;

  m.def("gpuinfo_json", &tk8s::gpuinfo_json, py::arg("with_links") = true, G());
  m.def(
      "hbm_write_probe",
      [](size_t bytes, int iters, const std::string& mode, int device, uint32_t value) {
        return tk8s::hbm_write_probe(bytes, iters, mode_of(mode), device, value);
      },
      py::arg("bytes"), py::arg("iters") = 10, py::arg("mode") = "nontemporal",
      py::arg("device") = 0, py::arg("value") = 0, G());
  m.def("md5_probe", &tk8s::md5_probe, py::arg("bytes"), py::arg("chunk_bytes") = 1024,
        py::arg("seed") = 0, py::arg("iters") = 10, py::arg("device") = 0, G());
  m.def("copy_probe", &tk8s::copy_probe, py::arg("src_device"), py::arg("dst_device"),
        py::arg("bytes"), py::arg("iters") = 10, py::arg("dma") = true, G());
  m.def(
      "rccl_allreduce",
      [](const std::vector<int>& devices, size_t min_bytes, size_t max_bytes, int factor,
         int iters, int warmup, const std::string& dtype, bool check) {
        tk8s::AllReduceConfig c;
        c.min_bytes = min_bytes;
        c.max_bytes = max_bytes;
        c.factor = factor;
        c.iters = iters;
        c.warmup = warmup;
        c.dtypes = {dtype_of(dtype)};
        c.check = check;
        return tk8s::allreduce_single_process(devices, c);
      },
      py::arg("devices"), py::arg("min_bytes") = 8, py::arg("max_bytes") = size_t(1) << 26,
      py::arg("factor") = 4, py::arg("iters") = 10, py::arg("warmup") = 2,
      py::arg("dtype") = "float32", py::arg("check") = true, G());
  m.def("rccl_version", &tk8s::rccl_version);
  m.def("allreduce_busbw", &tk8s::allreduce_busbw, py::arg("algbw_gbps"), py::arg("nranks"),
        "busbw of a ring all-reduce: algbw * 2(n-1)/n, 0 at n <= 1 (SURVEY.md N3)");
  m.def("release_probe_scratch", &tk8s::release_probe_scratch, G());

  // ---- raw launchers --------------------------------------------------------------------
  m.def("streaming_grid", &tk8s::streaming_grid, py::arg("blocks_per_cu") = 8);
  m.def(
      "hbm_fill",
      [](uintptr_t dst, size_t nbytes, uint32_t value, const std::string& mode, uintptr_t s) {
        tk8s::hbm_fill(ptr<void>(dst), nbytes, value, mode_of(mode), stream_of(s));
      },
      py::arg("dst"), py::arg("nbytes"), py::arg("value"), py::arg("mode") = "nontemporal",
      py::arg("stream") = 0);
  m.def(
      "verify_fill",
      [](uintptr_t src, size_t nbytes, uint32_t value, uintptr_t bad, uintptr_t s) {
        tk8s::verify_fill(ptr<const void>(src), nbytes, value, ptr<unsigned long long>(bad),
                          stream_of(s));
      },
      py::arg("src"), py::arg("nbytes"), py::arg("value"), py::arg("bad_words"),
      py::arg("stream") = 0);
  m.def(
      "philox_fill",
      [](uintptr_t dst, size_t nbytes, uint64_t seed, uintptr_t s) {
        tk8s::philox_fill(ptr<void>(dst), nbytes, seed, stream_of(s));
      },
      py::arg("dst"), py::arg("nbytes"), py::arg("seed"), py::arg("stream") = 0);
  m.def("md5_tree_workspace", &tk8s::md5_tree_workspace, py::arg("nbytes"),
        py::arg("chunk_bytes") = 1024);
  m.def(
      "md5_chunks",
      [](uintptr_t src, size_t nbytes, uint32_t chunk, uintptr_t digests, uintptr_t s) {
        tk8s::md5_chunks(ptr<const void>(src), nbytes, chunk, ptr<void>(digests), stream_of(s));
      },
      py::arg("src"), py::arg("nbytes"), py::arg("chunk_bytes"), py::arg("digests"),
      py::arg("stream") = 0);
  m.def(
      "md5_tree",
      [](uintptr_t src, size_t nbytes, uint32_t chunk, uintptr_t ws_a, uintptr_t ws_b,
         uintptr_t out16, uintptr_t s) {
        tk8s::md5_tree(ptr<const void>(src), nbytes, chunk, ptr<void>(ws_a), ptr<void>(ws_b),
                       ptr<void>(out16), stream_of(s));
      },
      py::arg("src"), py::arg("nbytes"), py::arg("chunk_bytes"), py::arg("ws_a"), py::arg("ws_b"),
      py::arg("out16"), py::arg("stream") = 0);
  m.def(
      "ar_fill",
      [](uintptr_t buf, size_t count, int rank, const std::string& dtype, uintptr_t s) {
        tk8s::ar_fill(ptr<void>(buf), count, rank, dtype_of(dtype), stream_of(s));
      },
      py::arg("buf"), py::arg("count"), py::arg("rank"), py::arg("dtype") = "float32",
      py::arg("stream") = 0);
  m.def(
      "ar_check",
      [](uintptr_t buf, size_t count, int nranks, const std::string& dtype, float tol,
         uintptr_t max_err_bits, uintptr_t bad, uintptr_t s) {
        tk8s::ar_check(ptr<const void>(buf), count, nranks, dtype_of(dtype), tol,
                       ptr<unsigned>(max_err_bits), ptr<unsigned long long>(bad), stream_of(s));
      },
      py::arg("buf"), py::arg("count"), py::arg("nranks"), py::arg("dtype") = "float32",
      py::arg("tol") = 0.0f, py::arg("max_err_bits") = 0, py::arg("bad") = 0,
      py::arg("stream") = 0);
  m.def(
      "stream_copy",
      [](uintptr_t dst, uintptr_t src, size_t nbytes, uintptr_t s) {
        tk8s::stream_copy(ptr<void>(dst), ptr<const void>(src), nbytes, stream_of(s));
      },
      py::arg("dst"), py::arg("src"), py::arg("nbytes"), py::arg("stream") = 0);
}
