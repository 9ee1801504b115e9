// N2 core: topology-aware GPU set selection (see topology.h).
#include "tk8s/topology.h"

#include <algorithm>
#include <limits>
#include <set>
#include <stdexcept>

namespace tk8s {

int link_weight(const std::string& type, int hops) {
  const int h = hops < 1 ? 1 : hops;
  if (type == "self") return 1000;
  if (type == "xgmi") return 100 / h;
  if (type == "pcie") return 10 / h > 0 ? 10 / h : 1;
  return 1;
}

namespace {

struct Score {
  int min_link;
  int64_t total;
};

Score score_set(int n, const std::vector<int>& w, const std::vector<int>& set) {
  if (set.size() < 2) return {0, 0};
  int mn = std::numeric_limits<int>::max();
  int64_t tot = 0;
  for (size_t a = 0; a < set.size(); ++a)
    for (size_t b = a + 1; b < set.size(); ++b) {
      // Symmetrise: a directed matrix may report different types per direction.
      const int v = std::min(w[set[a] * n + set[b]], w[set[b] * n + set[a]]);
      mn = std::min(mn, v);
      tot += v;
    }
  return {mn, tot};
}

bool better(const Score& s, const std::vector<int>& set, const Score& best,
            const std::vector<int>& best_set) {
  if (best_set.empty()) return true;
  if (s.min_link != best.min_link) return s.min_link > best.min_link;
  if (s.total != best.total) return s.total > best.total;
  return set < best_set;  // lexicographically smallest indices
}

double n_choose_k(size_t n, size_t k) {
  if (k > n) return 0;
  double r = 1;
  for (size_t i = 1; i <= k; ++i) r = r * (n - k + i) / i;
  return r;
}

}  // namespace

AllocationResult preferred_allocation(int n, const std::vector<int>& weights,
                                      const std::vector<int>& available,
                                      const std::vector<int>& must_include, int size) {
  if (n < 0 || static_cast<int64_t>(weights.size()) != static_cast<int64_t>(n) * n)
    throw std::invalid_argument("weights must be an n*n matrix");
  std::set<int> avail(available.begin(), available.end());
  std::set<int> must(must_include.begin(), must_include.end());
  for (int d : avail)
    if (d < 0 || d >= n) throw std::invalid_argument("available device index out of range");
  for (int d : must)
    if (!avail.count(d)) throw std::invalid_argument("must_include device not available");
  if (size < static_cast<int>(must.size()) || size > static_cast<int>(avail.size()) || size < 0)
    throw std::invalid_argument("requested size not satisfiable");

  std::vector<int> base(must.begin(), must.end());
  std::vector<int> cand;
  for (int d : avail)
    if (!must.count(d)) cand.push_back(d);
  const size_t need = static_cast<size_t>(size) - base.size();

  AllocationResult res;
  if (need == 0) {
    res.devices = base;
  } else if (n_choose_k(cand.size(), need) <= 2e5) {
    // Exhaustive: iterate combinations of `need` candidates in lexicographic order.
    std::vector<size_t> idx(need);
    for (size_t i = 0; i < need; ++i) idx[i] = i;
    Score best{0, 0};
    std::vector<int> best_set;
    while (true) {
      std::vector<int> set = base;
      for (size_t i : idx) set.push_back(cand[i]);
      std::sort(set.begin(), set.end());
      const Score s = score_set(n, weights, set);
      if (better(s, set, best, best_set)) {
        best = s;
        best_set = set;
      }
      // next combination
      size_t i = need;
      while (i > 0 && idx[i - 1] == cand.size() - need + (i - 1)) --i;
      if (i == 0) break;
      ++idx[i - 1];
      for (size_t j = i; j < need; ++j) idx[j] = idx[j - 1] + 1;
    }
    res.devices = best_set;
  } else {
    // Greedy: grow the set by the candidate with the strongest weakest-link to it.
    res.exhaustive = false;
    std::vector<int> set = base;
    std::vector<bool> used(n, false);
    for (int d : set) used[d] = true;
    while (set.size() < static_cast<size_t>(size)) {
      int pick = -1;
      Score ps{0, 0};
      for (int c : cand) {
        if (used[c]) continue;
        std::vector<int> trial = set;
        trial.push_back(c);
        std::sort(trial.begin(), trial.end());
        const Score s = score_set(n, weights, trial);
        if (pick < 0 || s.min_link > ps.min_link ||
            (s.min_link == ps.min_link && s.total > ps.total)) {
          pick = c;
          ps = s;
        }
      }
      used[pick] = true;
      set.push_back(pick);
    }
    std::sort(set.begin(), set.end());
    res.devices = set;
  }
  const Score s = score_set(n, weights, res.devices);
  res.min_link = s.min_link;
  res.total_link = s.total;
  return res;
}

}  // namespace tk8s
