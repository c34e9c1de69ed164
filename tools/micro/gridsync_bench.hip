// Microbenchmark: cost of one grid-wide barrier round (+ a 32 KB all-gather
// through global memory) in a persistent kernel on MI355X, to decide whether
// a persistent LSTM recurrence can beat one graph-replayed launch per step.
// Every spin is bounded: a block that waits too long sets an error flag and
// leaves, so the grid always drains.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/gridsync_bench.hip -o /tmp/gs
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ __launch_bounds__(256) void persist(float* buf, unsigned* cnt,
                                               int* err, float* out,
                                               int rounds) {
  const int G = gridDim.x;
  float acc = 0.f;
  for (int r = 0; r < rounds; ++r) {
    float* slot = buf + (r & 1) * G * 64;
    if (threadIdx.x < 64) slot[blockIdx.x * 64 + threadIdx.x] = r + threadIdx.x;
    __syncthreads();
    if (threadIdx.x == 0) {
      __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned target = static_cast<unsigned>(G) * (r + 1);
      long polls = 0;
      while (__hip_atomic_load(cnt, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
        if (++polls > (1l << 22)) { atomicExch(err, 1); break; }
      }
    }
    __syncthreads();
    if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
    // all-gather: every thread reads 32 floats of the other blocks' slices
    for (int k = 0; k < 32; ++k) acc += slot[(threadIdx.x * 32 + k * 7) % (G * 64)];
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

__global__ void noop() {}

int main() {
  float *buf, *out;
  unsigned* cnt;
  int* err;
  hipMalloc(&buf, 2 * 1024 * 64 * 4);
  hipMalloc(&out, 1024 * 256 * 4);
  hipMalloc(&cnt, 4);
  hipMalloc(&err, 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int G : {32, 64, 128, 256}) {
    const int R = 2000;
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
      hipMemset(cnt, 0, 4);
      hipMemset(err, 0, 4);
      hipEventRecord(a);
      hipLaunchKernelGGL(persist, dim3(G), dim3(256), 0, 0, buf, cnt, err, out, R);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      int e = 0;
      hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost);
      if (e) { printf("G=%d: barrier timed out\n", G); return 1; }
      if (ms < best) best = ms;
    }
    printf("persistent G=%4d: %.2f us per barrier round\n", G, 1e3f * best / R);
  }
  // dependent launches in a graph, for comparison
  hipStream_t s;
  hipStreamCreate(&s);
  hipGraph_t g;
  hipGraphExec_t ge;
  hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
  for (int i = 0; i < 200; ++i) hipLaunchKernelGGL(noop, dim3(64), dim3(256), 0, s);
  hipStreamEndCapture(s, &g);
  hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  hipGraphLaunch(ge, s);
  hipStreamSynchronize(s);
  hipEventRecord(a, s);
  for (int i = 0; i < 10; ++i) hipGraphLaunch(ge, s);
  hipEventRecord(b, s);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  printf("graph noop 64x256: %.2f us per launch\n", 1e3f * ms / 2000);
  return 0;
}
