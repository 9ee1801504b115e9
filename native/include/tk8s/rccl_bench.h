// N3: RCCL all-reduce validator (the "RCCL-tests DaemonSet" payload of BASELINE.json configs 4-5).
//
// Replaces the reference's only cluster health oracle — curl of the dashboard through the Rancher
// proxy (setup.sh:56-85) — with a data-plane check: every GPU worker must move real bytes over
// xGMI and produce the exact reduced value before the cluster is declared GPU-Ready.
//
// Two launch shapes:
//  * allreduce_single_process: one process drives n GPUs (one communicator of n ranks, all of
//    them local: a fresh unique id and the ranks' inits in one group).
//  * allreduce_rank_group: one process per NODE, driving all of that node's GPUs as consecutive
//    ranks of one multi-process communicator (ncclCommInitRankConfig per device inside one group).
//    On an 8-GPU node that is one runtime start instead of eight concurrent ones, each of which
//    would initialise all eight agents (the fabric Job's start-up cost).
//    allreduce_rank is the one-device case. Rank 0 creates the unique id and the caller ships it
//    to the other processes (file or control-plane KV, see tools/tk8s_rccl.cpp).
//
// Fail fast: the communicators are non-blocking (ncclConfig_t.blocking = 0), and
// every wait -- the init, each sweep point's collectives, each check -- polls the streams and
// ncclCommGetAsyncError under op_timeout_s. A timeout or an async error aborts every local
// communicator (ncclCommAbort) and returns {"ok":false,"phase":...,"error":...} at once, so a
// dead or hung peer costs one deadline, not the Job's whole wait.
//
// Bandwidth: algbw = bytes / time; busbw = algbw * 2(n-1)/n, the per-GPU
// link traffic of a ring all-reduce -- 0 at n = 1, where the "all-reduce" is a local copy and no
// fabric exists ("peak_busbw_gbps": null, "fabric": "1 GPU: no fabric").
#pragma once

#include <cstddef>
#include <functional>
#include <map>
#include <string>
#include <vector>

#include <rccl/rccl.h>

#include "tk8s/kernels.h"

namespace tk8s {

struct AllReduceConfig {
  size_t min_bytes = 8;
  size_t max_bytes = size_t(1) << 30;
  int factor = 2;        // size multiplier between sweep points
  int iters = 20;        // timed iterations per size
  int warmup = 5;        // untimed iterations per size
  std::vector<DType> dtypes{DType::kF32};  // one full sweep per dtype, on the same communicator
  bool check = true;     // run the N6 checker on the result of each size
  // free the communicators, streams and buffers before returning: a process that exits right
  // after (tk8s-rccl) skips it -- the driver reclaims all of it at exit, and ncclCommDestroy plus
  // the runtime's teardown were ~0.18 s of the fabric check's rank
  bool teardown = true;
  // bound on each wait (init, one sweep point, one check); <= 0: unbounded (blocking waits)
  double op_timeout_s = 20.0;
  // RCCL's blocking calls (TK8S_RCCL_BLOCKING=1): the init is then bounded only by the caller's
  // watchdog, not by an abort
  bool blocking = false;
  // called when a bounded wait starts (phase, its bound in s): the tool re-arms its watchdog
  std::function<void(const std::string&, double)> on_phase;
  // GPU-side fault point (TK8S_FAULTS rccl.hang@sweep / rccl.hang@check): stall the local ranks'
  // streams in that phase (kernels.h gpu_stall), as a rank whose GPU stopped would
  std::string stall_phase;
  // streams made ahead of the run (tk8s-rccl makes them while the unique id is exchanged), by
  // device; a device without one gets a fresh stream
  std::map<int, hipStream_t> streams;
};

std::string nccl_unique_id_hex(const ncclUniqueId& id);
bool nccl_unique_id_from_hex(const std::string& hex, ncclUniqueId* id);

// busbw of a ring all-reduce over n ranks for a given algbw: algbw * 2(n-1)/n (0 at n <= 1).
double allreduce_busbw(double algbw_gbps, int nranks);

// Returns {"ok":..,"mode":"single_process","nranks":n,"rccl_version":v,"sweep":{..},
// "results":[{dtype,bytes,count,time_us,algbw_gbps,busbw_gbps,max_err,bad}...],
// "peak_algbw_gbps":..,"peak_busbw_gbps":.. (null at n = 1)}; on failure {"ok":false,"phase":..}
std::string allreduce_single_process(const std::vector<int>& devices, const AllReduceConfig& cfg);

// Same record for ranks first_rank .. first_rank+devices.size()-1 of an nranks communicator,
// all driven by this process ("mode":"rank_group"; times are the slowest local rank's).
std::string allreduce_rank_group(int first_rank, int nranks, const std::vector<int>& devices,
                                 const ncclUniqueId& id, const AllReduceConfig& cfg);

// One rank of a multi-process communicator ("mode":"multi_process").
std::string allreduce_rank(int rank, int nranks, int device, const ncclUniqueId& id,
                           const AllReduceConfig& cfg);

int rccl_version();

}  // namespace tk8s
