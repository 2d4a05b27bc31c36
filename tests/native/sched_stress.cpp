// Concurrency / memory-safety stress of the GPU-slot scheduler (csrc/runtime/scheduler.cpp),
// built by tests/test_native_sanitizers.py with -fsanitize=address,undefined and, separately,
// -fsanitize=thread (the reference had real races — shared scratch files,
// a global PS/worker pair — and no sanitizer runs at all).
//
// 8 threads hammer submit/next/release/cancel/load/queued on one scheduler; invariants:
// per-GPU load never exceeds the slot count or goes negative, every admitted job is
// released exactly once, and the final state is empty.
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <thread>
#include <vector>

extern "C" {
void* csa_sched_create(int ngpu, int slots_per_gpu, int max_skip);
void csa_sched_destroy(void* h);
int csa_sched_submit(void* h, int64_t job, int ngpus);
int csa_sched_next(void* h, int64_t* job, int* gpus_out, int cap);
int csa_sched_release(void* h, int64_t job);
int csa_sched_cancel(void* h, int64_t job);
int csa_sched_load(void* h, int gpu);
int csa_sched_queued(void* h);
}

int main() {
  const int NG = 8, SLOTS = 3, THREADS = 8, OPS = 3000;
  void* s = csa_sched_create(NG, SLOTS, 4);
  std::atomic<int64_t> next_id{1};
  std::atomic<long> admitted{0}, released{0}, cancelled{0}, submitted{0};
  std::atomic<bool> bad{false};
  auto worker = [&](int tid) {
    std::mt19937 rng(1234 + tid);
    std::vector<int64_t> mine;
    for (int i = 0; i < OPS; ++i) {
      int r = rng() % 100;
      if (r < 30) {
        int64_t id = next_id++;
        if (csa_sched_submit(s, id, 1 + rng() % 3) == 0) submitted++;
      } else if (r < 70) {
        int64_t job;
        int gpus[NG];
        int n = csa_sched_next(s, &job, gpus, NG);
        if (n > 0) {
          admitted++;
          mine.push_back(job);
          for (int k = 0; k < n; ++k)
            if (gpus[k] < 0 || gpus[k] >= NG) bad = true;
        }
      } else if (r < 95) {
        if (!mine.empty()) {
          size_t k = rng() % mine.size();
          if (csa_sched_release(s, mine[k]) <= 0) bad = true;
          mine.erase(mine.begin() + k);
          released++;
        }
      } else {
        if (csa_sched_cancel(s, 1 + rng() % (next_id.load() + 1))) cancelled++;
      }
      for (int g = 0; g < NG; ++g) {
        int l = csa_sched_load(s, g);
        if (l < 0 || l > SLOTS) bad = true;
      }
      (void)csa_sched_queued(s);
    }
    for (int64_t j : mine) {
      if (csa_sched_release(s, j) <= 0) bad = true;
      released++;
    }
  };
  std::vector<std::thread> th;
  for (int t = 0; t < THREADS; ++t) th.emplace_back(worker, t);
  for (auto& t : th) t.join();
  // drain: admit and release everything left
  int64_t job;
  int gpus[NG];
  while (csa_sched_queued(s) > 0) {
    int n = csa_sched_next(s, &job, gpus, NG);
    if (n <= 0) { bad = true; break; }
    admitted++;
    csa_sched_release(s, job);
    released++;
  }
  for (int g = 0; g < NG; ++g)
    if (csa_sched_load(s, g) != 0) bad = true;
  if (admitted != released || admitted + cancelled != submitted) bad = true;
  csa_sched_destroy(s);
  std::printf("submitted=%ld admitted=%ld released=%ld cancelled=%ld ok=%d\n", (long)submitted, (long)admitted,
              (long)released, (long)cancelled, (int)!bad);
  return bad ? 1 : 0;
}
