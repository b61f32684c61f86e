// Native RCCL data plane: see rccl_comm.h.  The reference aggregates over torch.distributed.rpc (the server pulls
// every client's state dict and pushes the average back, `Server/dtds/distributed.py:794-823`); here every client
// rank joins one RCCL communicator and the aggregate is one in-place all-reduce of the flat parameter buffer, with
// the client weight folded into the collective (pre-multiplied sum).
#include "comm/rccl_comm.h"

#include <dlfcn.h>
#include <rccl/rccl.h>

#include <cstring>
#include <mutex>
#include <stdexcept>

namespace fedtgan {
namespace comm {
namespace {

struct Api {
  void* lib = nullptr;
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) comm_init_rank = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclRedOpCreatePreMulSum) premul_create = nullptr;
  decltype(&ncclRedOpDestroy) op_destroy = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
};

Api g_api;
std::mutex g_mu;
std::vector<ncclComm_t> g_comms;   // handle = index; destroyed slots are nullptr

template <typename F>
void resolve(F& fn, const char* name) {
  fn = reinterpret_cast<F>(dlsym(g_api.lib, name));
  if (!fn) throw std::runtime_error(std::string("rccl: missing symbol ") + name);
}

void check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess)
    throw std::runtime_error(std::string("rccl: ") + what + ": " + (g_api.error_string ? g_api.error_string(r) : "?"));
}

const Api& api() {
  if (!g_api.lib) throw std::runtime_error("rccl: library not loaded (rccl_load first)");
  return g_api;
}

ncclComm_t comm_of(int64_t h) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (h < 0 || h >= (int64_t)g_comms.size() || g_comms[(size_t)h] == nullptr)
    throw std::runtime_error("rccl: unknown communicator handle");
  return g_comms[(size_t)h];
}

}  // namespace

void rccl_load(const std::string& lib_path) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_api.lib) return;
  // the library torch already mapped (RTLD_NOLOAD): the same RCCL instance torch.distributed uses; else load it
  void* h = dlopen(lib_path.c_str(), RTLD_NOW | RTLD_NOLOAD);
  if (!h) h = dlopen(lib_path.c_str(), RTLD_NOW | RTLD_LOCAL);
  if (!h) throw std::runtime_error("rccl: cannot load " + lib_path + ": " + dlerror());
  g_api.lib = h;
  resolve(g_api.get_unique_id, "ncclGetUniqueId");
  resolve(g_api.comm_init_rank, "ncclCommInitRank");
  resolve(g_api.all_reduce, "ncclAllReduce");
  resolve(g_api.premul_create, "ncclRedOpCreatePreMulSum");
  resolve(g_api.op_destroy, "ncclRedOpDestroy");
  resolve(g_api.comm_destroy, "ncclCommDestroy");
  resolve(g_api.error_string, "ncclGetErrorString");
}

std::vector<uint8_t> rccl_unique_id() {
  ncclUniqueId id;
  check(api().get_unique_id(&id), "ncclGetUniqueId");
  std::vector<uint8_t> out(NCCL_UNIQUE_ID_BYTES);
  std::memcpy(out.data(), id.internal, NCCL_UNIQUE_ID_BYTES);
  return out;
}

int64_t rccl_init(const uint8_t* id, int rank, int nranks) {
  if (nranks < 1 || rank < 0 || rank >= nranks) throw std::runtime_error("rccl: bad rank / nranks");
  ncclUniqueId uid;
  std::memcpy(uid.internal, id, NCCL_UNIQUE_ID_BYTES);
  ncclComm_t c = nullptr;
  check(api().comm_init_rank(&c, nranks, uid, rank), "ncclCommInitRank");
  std::lock_guard<std::mutex> lk(g_mu);
  g_comms.push_back(c);
  return (int64_t)g_comms.size() - 1;
}

void rccl_all_reduce_f32(int64_t h, float* x, size_t count, float premul, hipStream_t s) {
  ncclComm_t c = comm_of(h);
  const Api& a = api();
  if (premul == 1.0f) {
    check(a.all_reduce(x, x, count, ncclFloat32, ncclSum, c, s), "ncclAllReduce");
    return;
  }
  // the scalar is read when the op is created (host immediate): a captured graph keeps this weight
  ncclRedOp_t op;
  check(a.premul_create(&op, &premul, ncclFloat32, ncclScalarHostImmediate, c), "ncclRedOpCreatePreMulSum");
  const ncclResult_t r = a.all_reduce(x, x, count, ncclFloat32, op, c, s);
  a.op_destroy(op, c);
  check(r, "ncclAllReduce");
}

void rccl_destroy(int64_t h) {
  ncclComm_t c = comm_of(h);
  {
    std::lock_guard<std::mutex> lk(g_mu);
    g_comms[(size_t)h] = nullptr;
  }
  check(api().comm_destroy(c), "ncclCommDestroy");
}

}  // namespace comm
}  // namespace fedtgan
