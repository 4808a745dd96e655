// Kernel-boundary cost on MI355X inside a hipGraph: N back-to-back launches of (a) an empty
// 1-workgroup kernel, (b) an empty 256-workgroup kernel, (c) 256 workgroups each writing 64 KB,
// (d) one launch that crosses N grid-wide barriers instead (atomic counter, agent-scope fences).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void k_empty() {}
__global__ void k_write(float* p, int n) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) p[i] = (float)i;
}
__global__ void k_barriers(unsigned* ctr, int nbar, float* p, int n) {
  for (int b = 0; b < nbar; ++b) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) p[i] += 1.f;
    __syncthreads();
    if (threadIdx.x == 0) {
      __threadfence();
      const unsigned target = (unsigned)(b + 1) * gridDim.x;
      atomicAdd(ctr, 1u);
      while (__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) __builtin_amdgcn_s_sleep(1);
    }
    __syncthreads();
  }
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <typename F>
float time_graph(hipStream_t s, F body, int reps = 20) {
  hipGraph_t g; hipGraphExec_t ge;
  hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
  body();
  hipStreamEndCapture(s, &g);
  hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  hipGraphLaunch(ge, s); hipStreamSynchronize(s);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0, s);
  for (int r = 0; r < reps; ++r) hipGraphLaunch(ge, s);
  hipEventRecord(e1, s); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  hipGraphExecDestroy(ge); hipGraphDestroy(g);
  return ms * 1000.f / reps;
}

int main() {
  hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const int N = 100, n = 256 * 16384;
  float* p; CK(hipMalloc(&p, n * sizeof(float)));
  unsigned* ctr; CK(hipMalloc(&ctr, sizeof(unsigned)));
  float t1 = time_graph(s, [&] { for (int i = 0; i < N; ++i) hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s); });
  float t2 = time_graph(s, [&] { for (int i = 0; i < N; ++i) hipLaunchKernelGGL(k_empty, dim3(256), dim3(512), 0, s); });
  float t3 = time_graph(s, [&] { for (int i = 0; i < N; ++i) hipLaunchKernelGGL(k_write, dim3(256), dim3(512), 0, s, p, n); });
  float t4 = time_graph(s, [&] {
    hipMemsetAsync(ctr, 0, sizeof(unsigned), s);
    hipLaunchKernelGGL(k_barriers, dim3(256), dim3(512), 0, s, ctr, N, p, n);
  });
  float t5 = time_graph(s, [&] {
    hipMemsetAsync(ctr, 0, sizeof(unsigned), s);
    hipLaunchKernelGGL(k_barriers, dim3(256), dim3(512), 0, s, ctr, 1, p, n);
  });
  printf("per launch in graph: empty 1 WG %.2f us | empty 256x512 %.2f us | 256 WGs writing 16 MB %.2f us\n",
         t1 / N, t2 / N, t3 / N);
  printf("grid barrier: one kernel with %d barriers (each after a 16 MB update pass) %.2f us/barrier; 1 barrier %.2f us total\n",
         N, (t4 - t5) / (N - 1), t5);
  return 0;
}
