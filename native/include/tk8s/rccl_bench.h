// N3: RCCL all-reduce validator (the "RCCL-tests DaemonSet" payload of BASELINE.json configs 4-5).
//
// Replaces the reference's only cluster health oracle — curl of the dashboard through the Rancher
// proxy (setup.sh:56-85) — with a data-plane check: every GPU worker must move real bytes over
// xGMI and produce the exact reduced value before the cluster is declared GPU-Ready.
//
// Two launch shapes:
//  * allreduce_single_process: one process drives n GPUs (ncclCommInitAll + group calls).
//  * allreduce_rank_group: one process per NODE, driving all of that node's GPUs as consecutive
//    ranks of one multi-process communicator (ncclCommInitRank per device inside one group).
//    On an 8-GPU node that is one runtime start instead of eight concurrent ones, each of which
//    would initialise all eight agents (the fabric Job's start-up cost).
//    allreduce_rank is the one-device case. Rank 0 creates the unique id and the caller ships it
//    to the other processes (file or control-plane KV, see tools/tk8s_rccl.cpp).
#pragma once

#include <cstddef>
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
  DType dtype = DType::kF32;
  bool check = true;     // run the N6 checker on the result of each size
  // free the communicators, streams and buffers before returning: a process that exits right
  // after (tk8s-rccl) skips it -- the driver reclaims all of it at exit, and ncclCommDestroy plus
  // the runtime's teardown were ~0.18 s of the fabric check's rank
  bool teardown = true;
};

std::string nccl_unique_id_hex(const ncclUniqueId& id);
bool nccl_unique_id_from_hex(const std::string& hex, ncclUniqueId* id);

// Returns {"ok":..,"mode":"single_process","nranks":n,"rccl_version":v,"results":[{bytes,count,
// time_us,algbw_gbps,busbw_gbps,max_err,bad}...],"peak_busbw_gbps":..}
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
