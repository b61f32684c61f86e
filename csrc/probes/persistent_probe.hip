// Kernel-boundary cost: a hipGraph of N empty kernels against ONE persistent kernel of N phases separated by a
// device-wide barrier (is a persistent multi-phase training step worth building?).
//
// The barrier is a monotone arrival counter in device memory: every workgroup's thread 0 publishes with an
// agent-scope release fetch-add (a vector atomic) and spins on an agent-scope acquire load until all of the
// grid has arrived for that phase.  The launch is cooperative (hipLaunchCooperativeKernel refuses a grid that
// cannot be co-resident), and every spin is bounded: a phase that does not complete within the spin budget
// sets an error flag and the kernel returns, so the grid always drains.
//
//   hipcc --offload-arch=gfx950 -O3 -o build/persistent_probe csrc/probes/persistent_probe.hip
//   build/persistent_probe [phases=25] [reps=200]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                       \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                    \
    }                                                                                  \
  } while (0)

__global__ void empty_kernel(float* sink) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && sink[0] < -1.f) sink[1] = 0.f;   // never true: keeps the launch
}

constexpr unsigned SPIN_LIMIT = 1u << 24;

__global__ void persistent_kernel(unsigned* arrive, unsigned* err, int phases, float* sink) {
  const unsigned n = gridDim.x;
  for (int p = 0; p < phases; ++p) {
    // (a phase's work would go here)
    if (threadIdx.x == 0 && sink[0] < -1.f) sink[1 + blockIdx.x] = (float)p;
    __syncthreads();
    if (threadIdx.x == 0) {
      __hip_atomic_fetch_add(arrive, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned target = (unsigned)(p + 1) * n;
      unsigned spins = 0;
      while (__hip_atomic_load(arrive, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > SPIN_LIMIT) {
          __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
    __syncthreads();
    if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
  }
}

static float time_graph(int blocks, int phases, int reps, float* sink, hipStream_t s) {
  hipGraph_t g;
  hipGraphExec_t ge;
  CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  for (int i = 0; i < phases; ++i) hipLaunchKernelGGL(empty_kernel, dim3(blocks), dim3(256), 0, s, sink);
  CHECK(hipStreamEndCapture(s, &g));
  CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int i = 0; i < 10; ++i) CHECK(hipGraphLaunch(ge, s));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  CHECK(hipEventRecord(a, s));
  for (int i = 0; i < reps; ++i) CHECK(hipGraphLaunch(ge, s));
  CHECK(hipEventRecord(b, s));
  CHECK(hipEventSynchronize(b));
  float ms = 0.f;
  CHECK(hipEventElapsedTime(&ms, a, b));
  CHECK(hipGraphExecDestroy(ge));
  CHECK(hipGraphDestroy(g));
  return ms * 1000.f / reps;   // us per graph
}

static float time_persistent(int blocks, int phases, int reps, unsigned* arrive, unsigned* err, float* sink,
                             hipStream_t s, bool* ok) {
  void* args[] = {&arrive, &err, &phases, &sink};
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  float total = 0.f;
  for (int i = 0; i < reps + 5; ++i) {
    CHECK(hipMemsetAsync(arrive, 0, sizeof(unsigned), s));
    CHECK(hipEventRecord(a, s));
    hipError_t e = hipLaunchCooperativeKernel(reinterpret_cast<const void*>(persistent_kernel), dim3(blocks), dim3(256),
                                              args, 0, s);
    if (e != hipSuccess) {
      std::fprintf(stderr, "cooperative launch of %d workgroups refused: %s\n", blocks, hipGetErrorString(e));
      *ok = false;
      return 0.f;
    }
    CHECK(hipEventRecord(b, s));
    CHECK(hipEventSynchronize(b));
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, a, b));
    if (i >= 5) total += ms;
  }
  unsigned herr = 0;
  CHECK(hipMemcpy(&herr, err, sizeof(unsigned), hipMemcpyDeviceToHost));
  *ok = herr == 0;
  return total * 1000.f / reps;   // us per launch
}

int main(int argc, char** argv) {
  const int phases = argc > 1 ? std::atoi(argv[1]) : 25;
  const int reps = argc > 2 ? std::atoi(argv[2]) : 200;
  hipStream_t s;
  CHECK(hipStreamCreate(&s));
  unsigned *arrive, *err;
  float* sink;
  CHECK(hipMalloc(&arrive, sizeof(unsigned)));
  CHECK(hipMalloc(&err, sizeof(unsigned)));
  CHECK(hipMalloc(&sink, (1 + 4096) * sizeof(float)));
  CHECK(hipMemset(err, 0, sizeof(unsigned)));
  CHECK(hipMemset(sink, 0, (1 + 4096) * sizeof(float)));
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  std::printf("device %s, %d CUs; %d phases, %d reps\n", prop.name, prop.multiProcessorCount, phases, reps);
  for (int blocks : {256, 1024}) {
    const float g1 = time_graph(blocks, 1, reps, sink, s);
    const float gn = time_graph(blocks, phases, reps, sink, s);
    bool ok1 = true, okn = true;
    const float p1 = time_persistent(blocks, 1, reps, arrive, err, sink, s, &ok1);
    const float pn = time_persistent(blocks, phases, reps, arrive, err, sink, s, &okn);
    std::printf("{\"workgroups\": %d, \"graph_us_per_kernel\": %.3f, \"graph_us_total\": %.2f, "
                "\"persistent_us_per_boundary\": %.3f, \"persistent_us_total\": %.2f, \"barrier_ok\": %s}\n",
                blocks, (gn - g1) / (phases - 1), gn, okn ? (pn - p1) / (phases - 1) : -1.f, pn,
                (ok1 && okn) ? "true" : "false");
  }
  CHECK(hipFree(arrive));
  CHECK(hipFree(err));
  CHECK(hipFree(sink));
  return 0;
}
