// Host-only self-test of the native pieces that do not need a GPU, built with
// -fsanitize=address,undefined by tests/test_sanitizers.py (sanitizers on host
// code). Exercises the xGMI-aware allocator (topology.cpp), the JSON writer (common.h) and the
// CLI argument parser (tools/args.h) with valid and hostile inputs. Exit 0 = all checks passed.
#include <cstdio>
#include <stdexcept>
#include <string>
#include <vector>

#include "../tools/args.h"
#include "tk8s/json.h"
#include "tk8s/topology.h"

namespace {

int failures = 0;

void check(bool ok, const char* what) {
  if (!ok) {
    std::fprintf(stderr, "FAIL: %s\n", what);
    ++failures;
  }
}

std::vector<int> islands(int n, int split) {
  std::vector<int> w(n * n);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j)
      w[i * n + j] = i == j ? 1000 : ((i < split) == (j < split) ? 100 : 10);
  return w;
}

}  // namespace

int main() {
  // allocator: best set on one island, must_include honoured, every size on 8 GPUs
  const auto w = islands(8, 4);
  auto r = tk8s::preferred_allocation(8, w, {2, 3, 4, 5, 6, 7}, {}, 4);
  check(r.devices == std::vector<int>({4, 5, 6, 7}), "island selection");
  r = tk8s::preferred_allocation(8, w, {0, 1, 2, 3, 4, 5, 6, 7}, {6}, 2);
  check(r.devices.size() == 2 && (r.devices[0] == 6 || r.devices[1] == 6), "must_include");
  for (int k = 1; k <= 8; ++k) {
    std::vector<int> all = {0, 1, 2, 3, 4, 5, 6, 7};
    r = tk8s::preferred_allocation(8, w, all, {}, k);
    check(static_cast<int>(r.devices.size()) == k, "size k");
  }
  // a 64-GPU request exercises the greedy fallback path
  std::vector<int> big(64 * 64, 100), all64;
  for (int i = 0; i < 64; ++i) {
    big[i * 64 + i] = 1000;
    all64.push_back(i);
  }
  r = tk8s::preferred_allocation(64, big, all64, {}, 32);
  check(r.devices.size() == 32, "greedy fallback size");
  // hostile inputs must throw, never read out of bounds
  int threw = 0;
  try { tk8s::preferred_allocation(8, std::vector<int>(10), {0}, {}, 1); } catch (const std::invalid_argument&) { ++threw; }
  try { tk8s::preferred_allocation(8, w, {0, 99}, {}, 1); } catch (const std::invalid_argument&) { ++threw; }
  try { tk8s::preferred_allocation(8, w, {0, 1}, {5}, 1); } catch (const std::invalid_argument&) { ++threw; }
  try { tk8s::preferred_allocation(8, w, {0, 1}, {}, 3); } catch (const std::invalid_argument&) { ++threw; }
  try { tk8s::preferred_allocation(-1, {}, {}, {}, 1); } catch (const std::invalid_argument&) { ++threw; }
  check(threw == 5, "invalid inputs throw");
  check(tk8s::link_weight("xgmi", 0) == 100 && tk8s::link_weight("pcie", 100) == 1, "link weights");

  // argument parser
  const char* argv[] = {"prog", "--iters", "3", "--flag", "--out=x.json", "--neg", "-5"};
  tk8s::Args a(7, const_cast<char**>(argv));
  check(a.num("iters", 0) == 3 && a.has("flag") && a.str("out") == "x.json", "args");
  check(a.str("neg") == "-5", "negative value");
  int bad = 0;
  try {
    const char* argv2[] = {"prog", "stray"};
    tk8s::Args b(2, const_cast<char**>(argv2));
  } catch (const std::invalid_argument&) {
    ++bad;
  }
  check(bad == 1, "stray argument rejected");

  // JSON writer: escaping, and doubles that keep their precision -- a wall-clock timestamp in ms
  // (~1.8e12) must not be rounded to whole seconds (the RCCL ranks' init spread is a difference
  // of two of them)
  const std::string j = tk8s::Json().kv("s", std::string("a\"b\\c\n")).kv("t", 1760000000123.456).kv("x", 0.174566)
                            .kv("n", static_cast<int64_t>(-3)).str();
  check(j == "{\"s\":\"a\\\"b\\\\c\\n\",\"t\":1760000000123.456,\"x\":0.174566,\"n\":-3}", "json writer");
  if (failures) {
    std::fprintf(stderr, "json: %s\n", j.c_str());
    return 1;
  }
  std::printf("host selftest ok\n");
  return 0;
}
