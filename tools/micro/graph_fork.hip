// Do hipGraph replays run forked branches concurrently, and does a CU-masked
// stream keep its mask under capture?  Branch A: 200 dependent 1-block
// kernels (latency chain, like the LSTM steps).  Branch B: one long
// busy-loop kernel over G blocks (like a persistent conv kernel).
//   hipcc --offload-arch=gfx950 -O3 tools/micro/graph_fork.hip -o tools/micro/graph_fork
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); return 1; } } while (0)

__global__ void step(float* h) {
  float v = h[threadIdx.x];
  for (int i = 0; i < 64; ++i) v = v * 0.999f + 0.001f;
  h[threadIdx.x] = v;
}

__global__ __launch_bounds__(256) void busy(float* o, int iters) {
  float v = threadIdx.x;
  for (int i = 0; i < iters; ++i) v = __builtin_fmaf(v, 0.9999f, 0.0001f);
  o[blockIdx.x * 256 + threadIdx.x] = v;
}

static float time_graph(hipGraphExec_t ge, hipStream_t s) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipGraphLaunch(ge, s);
  hipStreamSynchronize(s);
  hipEventRecord(a, s);
  for (int i = 0; i < 5; ++i) hipGraphLaunch(ge, s);
  hipEventRecord(b, s);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms / 5;
}

int main(int argc, char** argv) {
  float *h, *o;
  CK(hipMalloc(&h, 256 * 4));
  CK(hipMalloc(&o, 4096 * 256 * 4));
  CK(hipMemset(h, 0, 1024));
  hipStream_t s0, s1, sm;
  CK(hipStreamCreate(&s0));
  CK(hipStreamCreate(&s1));
  // CU mask: first half of the CUs (bits 0..127) for the busy stream
  std::vector<uint32_t> mask(8, 0u);
  for (int i = 0; i < 4; ++i) mask[i] = 0xffffffffu;
  CK(hipExtStreamCreateWithCUMask(&sm, 8, mask.data()));
  hipEvent_t fork, join;
  CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
  const int iters = 200000;
  for (int G : {128, 256, 512, 1024}) {
    for (int mode = 0; mode < 4; ++mode) {
      // 0: chain only, 1: busy only, 2: serial, 3: forked
      hipStream_t bs = (argc > 1) ? sm : s1;
      hipGraph_t g;
      hipGraphExec_t ge;
      CK(hipStreamBeginCapture(s0, hipStreamCaptureModeGlobal));
      if (mode == 3) {
        CK(hipEventRecord(fork, s0));
        CK(hipStreamWaitEvent(bs, fork, 0));
        hipLaunchKernelGGL(busy, dim3(G), dim3(256), 0, bs, o, iters);
        CK(hipEventRecord(join, bs));
      }
      if (mode != 1)
        for (int i = 0; i < 200; ++i) hipLaunchKernelGGL(step, dim3(1), dim3(64), 0, s0, h);
      if (mode == 1 || mode == 2)
        hipLaunchKernelGGL(busy, dim3(G), dim3(256), 0, s0, o, iters);
      if (mode == 3) CK(hipStreamWaitEvent(s0, join, 0));
      CK(hipStreamEndCapture(s0, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      float ms = time_graph(ge, s0);
      const char* names[] = {"chain", "busy", "serial", "forked"};
      printf("G=%4d %-7s %s: %.3f ms\n", G, names[mode], argc > 1 ? "cumask" : "plain", ms);
      hipGraphExecDestroy(ge);
      hipGraphDestroy(g);
    }
  }
  // eager forked for comparison
  for (int G : {256, 1024}) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipStream_t bs = (argc > 1) ? sm : s1;
    hipDeviceSynchronize();
    hipEventRecord(a, s0);
    hipEventRecord(fork, s0);
    hipStreamWaitEvent(bs, fork, 0);
    hipLaunchKernelGGL(busy, dim3(G), dim3(256), 0, bs, o, iters);
    hipEventRecord(join, bs);
    for (int i = 0; i < 200; ++i) hipLaunchKernelGGL(step, dim3(1), dim3(64), 0, s0, h);
    hipStreamWaitEvent(s0, join, 0);
    hipEventRecord(b, s0);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    printf("G=%4d eager forked %s: %.3f ms\n", G, argc > 1 ? "cumask" : "plain", ms);
  }
  return 0;
}
