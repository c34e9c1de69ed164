// Phase timing of learner_head_fwd (block 0, s_memtime deltas).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -munsafe-fp-atomics -Icsrc \
//     tools/micro/head_trace.hip -o tools/micro/head_trace
#define SA_HEAD_TRACE 1
#include "kernels/learner_io.hip"

#include <cstdio>
#include <vector>

int main() {
  const int A = 9, B = 32, T = 100, T1 = T + 1;
  float *core, *wp, *bp, *wb, *bb, *beh, *rew, *dl, *dv, *part, *loss;
  int64_t* act;
  uint8_t* done;
  unsigned* ticket;
  hipMalloc(&core, sizeof(float) * T1 * B * 256);
  hipMalloc(&wp, sizeof(float) * 256 * A);
  hipMalloc(&bp, sizeof(float) * A);
  hipMalloc(&wb, sizeof(float) * 256);
  hipMalloc(&bb, sizeof(float));
  hipMalloc(&beh, sizeof(float) * T1 * B * A);
  hipMalloc(&rew, sizeof(float) * T1 * B);
  hipMalloc(&act, sizeof(int64_t) * T1 * B);
  hipMalloc(&done, T1 * B);
  hipMalloc(&dl, sizeof(float) * T * B * A);
  hipMalloc(&dv, sizeof(float) * T * B);
  hipMalloc(&part, sizeof(float) * 3 * B);
  hipMalloc(&loss, sizeof(float) * 4);
  hipMalloc(&ticket, 4);
  hipMemset(core, 0, sizeof(float) * T1 * B * 256);
  hipMemset(wp, 0, sizeof(float) * 256 * A);
  hipMemset(bp, 0, sizeof(float) * A);
  hipMemset(wb, 0, sizeof(float) * 256);
  hipMemset(bb, 0, sizeof(float));
  hipMemset(beh, 0, sizeof(float) * T1 * B * A);
  hipMemset(rew, 0, sizeof(float) * T1 * B);
  hipMemset(act, 0, sizeof(int64_t) * T1 * B);
  hipMemset(done, 0, T1 * B);
  hipMemset(ticket, 0, 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int rep = 0; rep < 4; ++rep) {
    hipEventRecord(a);
    sa::learner_head_fwd_launch(core, wp, bp, wb, bb, beh, act, rew, done, T, B, A,
                                0.99f, 0, 1.f, 1.f, 0.5f, 0.01f, dl, dv, part, ticket,
                                loss, 0);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    unsigned long long tr[16];
    hipMemcpyFromSymbol(tr, HIP_SYMBOL(sa::sa_head_trace), sizeof(tr));
    printf("rep %d: %.1f us total; phase clocks:", rep, ms * 1e3f);
    for (int i = 1; i <= 8; ++i) printf(" %llu", tr[i] - tr[i - 1]);
    printf("\n");
  }
  return 0;
}
