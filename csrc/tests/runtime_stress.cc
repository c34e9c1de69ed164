// Concurrency stress of the host runtime, built with -fsanitize=thread or
// -fsanitize=address,undefined by tests/test_sanitizers.py (SURVEY.md §5.2:
// the reference has only compile-time lock annotations; here the dynamic
// batcher and the shared-memory trajectory ring also run under TSan/ASan).
//
//   batcher: 16 client threads x N Compute() calls (value -> 2 * value), two
//            server threads completing batches out of order with random
//            delays, then Close() while servers still wait.
//   ring:    4 producer threads x M slots, one consumer thread draining in
//            batches, payload checksums verified, then Close().
// Exit code 0 = all results correct (sanitizer findings abort with their own
// exit code).
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <unistd.h>
#include <vector>

#include "batcher/batcher.h"
#include "envpool/shm_ring.h"

namespace {

int fail(const char* what) {
  std::fprintf(stderr, "FAIL: %s\n", what);
  return 1;
}

int batcher_stress(int per_client) {
  sa::Batcher b(1, 8, 5);
  std::atomic<int> bad{0};
  std::atomic<bool> stop{false};
  auto server = [&](int seed) {
    std::mt19937 rng(seed);
    while (!stop.load()) {
      std::vector<sa::OwnedTensor> in;
      int64_t id = 0;
      sa::Status s = b.GetInputs(&in, &id);
      if (!s.ok()) return;  // closed
      sa::OwnedTensor out = sa::OwnedTensor::Alloc(in[0].meta);
      const float* x = reinterpret_cast<const float*>(in[0].data.get());
      float* y = reinterpret_cast<float*>(out.data.get());
      const size_t n = in[0].meta.nbytes() / sizeof(float);
      for (size_t i = 0; i < n; ++i) y[i] = 2.f * x[i];
      if (rng() % 4 == 0) std::this_thread::sleep_for(std::chrono::microseconds(rng() % 200));
      sa::TensorView v{out.meta, out.data.get()};
      if (!b.SetOutputs({v}, id).ok()) return;
    }
  };
  auto client = [&](int c) {
    for (int i = 0; i < per_client; ++i) {
      float x[4] = {float(c), float(i), float(c * 1000 + i), -1.f};
      sa::TensorMeta m{"<f4", 4, {1, 4}};
      std::vector<sa::OwnedTensor> out;
      sa::Status s = b.Compute({sa::TensorView{m, x}}, &out);
      if (!s.ok() || out.size() != 1) { bad++; continue; }
      const float* y = reinterpret_cast<const float*>(out[0].data.get());
      for (int k = 0; k < 4; ++k)
        if (y[k] != 2.f * x[k]) bad++;
    }
  };
  std::vector<std::thread> ts;
  ts.emplace_back(server, 1);
  ts.emplace_back(server, 2);
  std::vector<std::thread> cs;
  for (int c = 0; c < 16; ++c) cs.emplace_back(client, c);
  for (auto& t : cs) t.join();
  stop = true;
  b.Close();
  for (auto& t : ts) t.join();
  if (bad.load() != 0) return fail("batcher results");
  if (b.num_requests() != 16LL * per_client) return fail("batcher request count");
  return 0;
}

int ring_stress(int per_producer) {
  const std::string name = "/sa_stress_" + std::to_string(::getpid());
  sa::ShmRing ring(name, 8, 4096, true);
  std::atomic<int> bad{0};
  std::atomic<long> consumed{0};
  auto producer = [&](int p) {
    for (int i = 0; i < per_producer; ++i) {
      const int64_t s = ring.AcquireWrite(5000);
      if (s < 0) { bad++; return; }
      uint32_t* d = reinterpret_cast<uint32_t*>(ring.slot_data(s));
      const uint32_t key = static_cast<uint32_t>(p * 100000 + i);
      for (int k = 0; k < 1024; ++k) d[k] = key ^ static_cast<uint32_t>(k * 2654435761u);
      ring.Commit(s);
    }
  };
  std::thread consumer([&]() {
    const long total = 4L * per_producer;
    int64_t got[8];
    while (consumed.load() < total) {
      const int64_t n = ring.AcquireReadMany(4, got, 5000);
      if (n <= 0) { bad++; return; }
      for (int64_t j = 0; j < n; ++j) {
        const uint32_t* d = reinterpret_cast<const uint32_t*>(ring.slot_data(got[j]));
        const uint32_t key = d[0];
        for (int k = 0; k < 1024; ++k)
          if (d[k] != (key ^ static_cast<uint32_t>(k * 2654435761u))) { bad++; break; }
        ring.Release(got[j]);
      }
      consumed += n;
    }
  });
  std::vector<std::thread> ps;
  for (int p = 0; p < 4; ++p) ps.emplace_back(producer, p);
  for (auto& t : ps) t.join();
  consumer.join();
  ring.Close();
  sa::ShmRing::Unlink(name);
  if (bad.load() != 0) return fail("ring payloads");
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 200;
  int rc = batcher_stress(n);
  if (rc == 0) rc = ring_stress(n);
  if (rc == 0) std::printf("runtime stress ok\n");
  return rc;
}
