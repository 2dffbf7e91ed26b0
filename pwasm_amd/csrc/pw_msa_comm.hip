// pw_msa_comm.hip — the GapAssem histogram collectives over RCCL.
//
// With the rows of a layout sharded over GPUs, each rank's pw_msa_count leaves
// partial column histograms counts[n_cols][6] and its bounds minmax[0..2].  The merge is one
// grouped RCCL call set over xGMI: a SUM all-reduce of the int32 histograms (integer sums are
// order-independent: bit-identical to a single-GPU count) plus MIN / MAX all-reduces of the
// bounds.  The reduce-scatter variant leaves each rank the merged counts of its own column
// range only (1/N of the all-reduce's receive traffic) for a column-sharded bestChar.
//
// librccl is opened on first use (dlopen): the product library carries no link-time dependency
// on it, and single-GPU callers never load it.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <limits.h>
#include <rccl/rccl.h>
#include <string.h>

#include <mutex>

#include "pwasm_amd.h"

namespace {

struct Rccl {
  bool ok = false;
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) comm_init_rank = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclReduceScatter) reduce_scatter = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
};

const Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return;
    r.get_unique_id = (decltype(r.get_unique_id))dlsym(h, "ncclGetUniqueId");
    r.comm_init_rank = (decltype(r.comm_init_rank))dlsym(h, "ncclCommInitRank");
    r.comm_destroy = (decltype(r.comm_destroy))dlsym(h, "ncclCommDestroy");
    r.all_reduce = (decltype(r.all_reduce))dlsym(h, "ncclAllReduce");
    r.reduce_scatter = (decltype(r.reduce_scatter))dlsym(h, "ncclReduceScatter");
    r.all_gather = (decltype(r.all_gather))dlsym(h, "ncclAllGather");
    r.group_start = (decltype(r.group_start))dlsym(h, "ncclGroupStart");
    r.group_end = (decltype(r.group_end))dlsym(h, "ncclGroupEnd");
    r.ok = r.get_unique_id && r.comm_init_rank && r.comm_destroy && r.all_reduce && r.reduce_scatter && r.all_gather &&
           r.group_start && r.group_end;
  });
  return r;
}

// minmax[2] (first out-of-range row, local) -> global row index before the MIN reduction
__global__ void rebase_bad_row(int32_t* minmax, uint32_t row_base) {
  if (threadIdx.x == 0 && minmax[2] != INT_MAX) minmax[2] += (int32_t)row_base;
}

}  // namespace

extern "C" int pw_comm_unique_id(uint8_t* id) {
  const Rccl& r = rccl();
  if (!r.ok) return PW_E_HIP;
  if (!id) return PW_E_ARG;
  ncclUniqueId u;
  if (r.get_unique_id(&u) != ncclSuccess) return PW_E_HIP;
  memcpy(id, u.internal, PW_COMM_ID_BYTES);
  return PW_OK;
}

extern "C" int pw_comm_init(void** comm, int nranks, const uint8_t* id, int rank) {
  const Rccl& r = rccl();
  if (!r.ok) return PW_E_HIP;
  if (!comm || !id || nranks < 1 || rank < 0 || rank >= nranks) return PW_E_ARG;
  ncclUniqueId u;
  memcpy(u.internal, id, PW_COMM_ID_BYTES);
  ncclComm_t c = nullptr;
  if (r.comm_init_rank(&c, nranks, u, rank) != ncclSuccess) return PW_E_HIP;
  *comm = c;
  return PW_OK;
}

extern "C" int pw_comm_destroy(void* comm) {
  const Rccl& r = rccl();
  if (!r.ok) return PW_E_HIP;
  if (!comm) return PW_E_ARG;
  return r.comm_destroy((ncclComm_t)comm) == ncclSuccess ? PW_OK : PW_E_HIP;
}

extern "C" int pw_msa_counts_allreduce(const pw_msa_args* a, uint32_t row_base, void* comm, void* stream) {
  const Rccl& r = rccl();
  if (!r.ok) return PW_E_HIP;
  if (!a || !a->counts || !a->minmax || a->n_cols <= 0 || !comm) return PW_E_ARG;
  hipStream_t s = (hipStream_t)stream;
  ncclComm_t c = (ncclComm_t)comm;
  hipLaunchKernelGGL(rebase_bad_row, dim3(1), dim3(64), 0, s, a->minmax, row_base);
  if (hipGetLastError() != hipSuccess) return PW_E_HIP;
  int32_t* mm = a->minmax;
  bool ok = r.group_start() == ncclSuccess;
  ok = ok && r.all_reduce(a->counts, a->counts, (size_t)a->n_cols * 6, ncclInt32, ncclSum, c, s) == ncclSuccess;
  ok = ok && r.all_reduce(mm, mm, 1, ncclInt32, ncclMin, c, s) == ncclSuccess;      // mincol
  ok = ok && r.all_reduce(mm + 1, mm + 1, 1, ncclInt32, ncclMax, c, s) == ncclSuccess;  // maxcol
  ok = ok && r.all_reduce(mm + 2, mm + 2, 1, ncclInt32, ncclMin, c, s) == ncclSuccess;  // first bad row
  ok = (r.group_end() == ncclSuccess) && ok;
  return ok ? PW_OK : PW_E_HIP;
}

extern "C" int pw_msa_counts_reduce_scatter(const int32_t* counts, int32_t* counts_part, uint64_t cols_per_rank,
                                            void* comm, void* stream) {
  const Rccl& r = rccl();
  if (!r.ok) return PW_E_HIP;
  if (!counts || !counts_part || !comm || cols_per_rank == 0) return PW_E_ARG;
  return r.reduce_scatter(counts, counts_part, (size_t)cols_per_rank * 6, ncclInt32, ncclSum, (ncclComm_t)comm,
                          (hipStream_t)stream) == ncclSuccess
             ? PW_OK
             : PW_E_HIP;
}

// Column-sharded bestChar: reduce-scatter of the row-sharded histograms by column
// range + the bounds, bestChar and the zero-coverage scan of the rank's range, all-gather of the
// consensus ranges (in place) + MIN of the first zero column.
extern "C" int pw_msa_call_sharded(const pw_msa_args* a, uint32_t row_base, int32_t* counts_part,
                                   uint64_t cols_per_rank, int rank, int nranks, void* comm, void* stream) {
  const Rccl& r = rccl();
  if (!r.ok) return PW_E_HIP;
  if (!a || !a->counts || !a->consensus || !a->minmax || a->n_cols <= 0 || !comm || !counts_part || nranks < 1 ||
      rank < 0 || rank >= nranks || cols_per_rank * (uint64_t)nranks < (uint64_t)a->n_cols)
    return PW_E_ARG;
  hipStream_t s = (hipStream_t)stream;
  ncclComm_t c = (ncclComm_t)comm;
  hipLaunchKernelGGL(rebase_bad_row, dim3(1), dim3(64), 0, s, a->minmax, row_base);
  if (hipGetLastError() != hipSuccess) return PW_E_HIP;
  int32_t* mm = a->minmax;
  bool ok = r.group_start() == ncclSuccess;
  ok = ok && r.reduce_scatter(a->counts, counts_part, (size_t)cols_per_rank * 6, ncclInt32, ncclSum, c, s) == ncclSuccess;
  ok = ok && r.all_reduce(mm, mm, 1, ncclInt32, ncclMin, c, s) == ncclSuccess;
  ok = ok && r.all_reduce(mm + 1, mm + 1, 1, ncclInt32, ncclMax, c, s) == ncclSuccess;
  ok = ok && r.all_reduce(mm + 2, mm + 2, 1, ncclInt32, ncclMin, c, s) == ncclSuccess;
  ok = (r.group_end() == ncclSuccess) && ok;
  if (!ok) return PW_E_HIP;
  const uint64_t lo = (uint64_t)rank * cols_per_rank;
  const int32_t c_lo = (int32_t)(lo < (uint64_t)a->n_cols ? lo : (uint64_t)a->n_cols);
  const int32_t c_hi = (int32_t)(lo + cols_per_rank < (uint64_t)a->n_cols ? lo + cols_per_rank : (uint64_t)a->n_cols);
  const int rc = pw_msa_call_cols(a, c_lo, c_hi, counts_part, stream);
  if (rc != PW_OK) return rc;
  ok = r.group_start() == ncclSuccess;
  ok = ok && r.all_gather(a->consensus + lo, a->consensus, cols_per_rank, ncclUint8, c, s) == ncclSuccess;
  ok = ok && r.all_reduce(mm + 3, mm + 3, 1, ncclInt32, ncclMin, c, s) == ncclSuccess;
  ok = (r.group_end() == ncclSuccess) && ok;
  return ok ? PW_OK : PW_E_HIP;
}
