// Native RCCL data plane (csrc/comm): the federated round's weight all-reduce issued from C++ on the caller's HIP
// stream.  It is graph-capturable and has no ProcessGroup bookkeeping (work objects, watchdog, stream hand-offs).
// RCCL is the instance torch already loaded (its librccl.so, dlopen'ed by path): one RCCL per process, whichever
// plane a collective goes through.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstdint>
#include <string>
#include <vector>

namespace fedtgan {
namespace comm {

void rccl_load(const std::string& lib_path);                        // dlopen + resolve the entry points (once)
std::vector<uint8_t> rccl_unique_id();                              // ncclGetUniqueId: 128 opaque bytes
int64_t rccl_init(const uint8_t* id, int rank, int nranks);         // ncclCommInitRank on the current device
// x <- sum over ranks of premul * x_rank (premul == 1: a plain sum), fp32, on stream s
void rccl_all_reduce_f32(int64_t comm, float* x, size_t count, float premul, hipStream_t s);
void rccl_destroy(int64_t comm);

}  // namespace comm
}  // namespace fedtgan
