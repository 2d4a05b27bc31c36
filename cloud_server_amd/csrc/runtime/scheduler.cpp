// GPU-slot scheduler for the multi-tenant job runtime (host C++, C ABI via ctypes).
//
// Reference: there was exactly one PS container and one worker container cluster-wide
// (global_settings.py:15-20) and every launch began with `pkill -9 python` inside the PS
// (apps/construction/views.py:128-129), i.e. one training job at a time and a new job
// killed the running one.  On an 8x MI355X node the sample model uses a tiny fraction of
// one GPU, so the throughput lever is packing many independent jobs:
//
//   * every GPU exposes `slots_per_gpu` slots (jobs sharing a GPU run on separate HIP
//     streams in separate processes),
//   * a job asks for `ngpus` (1 = single-GPU job, >1 = a data-parallel job that needs
//     `ngpus` distinct GPUs, one rank per GPU),
//   * placement = least-loaded GPUs first (ties -> lowest id), FIFO admission with
//     head-of-line skipping limited by `max_skip` so a wide job is not starved forever,
//   * the scheduler is thread-safe (one mutex); tests/native/ stress it under ASan/UBSan
//     and ThreadSanitizer.
//
// The Python job manager (runtime/scheduler.py) wraps this library and falls back to a
// pure-Python implementation of the same policy if the .so is unavailable.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <deque>
#include <mutex>
#include <vector>

namespace {

struct Pending {
  int64_t job;
  int ngpus;
  int skipped;
};

struct Sched {
  int ngpu = 0;
  int slots_per_gpu = 1;
  int max_skip = 8;
  std::vector<int> load;                      // running jobs per GPU
  std::vector<std::vector<int64_t>> owners;   // job ids per GPU
  std::deque<Pending> queue;
  std::mutex mu;
};

// choose `n` distinct GPUs with a free slot, least loaded first; empty if impossible
std::vector<int> pick(Sched& s, int n) {
  std::vector<int> idx;
  for (int g = 0; g < s.ngpu; ++g)
    if (s.load[g] < s.slots_per_gpu) idx.push_back(g);
  if ((int)idx.size() < n) return {};
  std::stable_sort(idx.begin(), idx.end(), [&](int a, int b) { return s.load[a] < s.load[b]; });
  idx.resize(n);
  std::sort(idx.begin(), idx.end());
  return idx;
}

void place(Sched& s, int64_t job, const std::vector<int>& gpus) {
  for (int g : gpus) {
    s.load[g]++;
    s.owners[g].push_back(job);
  }
}

}  // namespace

extern "C" {

void* csa_sched_create(int ngpu, int slots_per_gpu, int max_skip) {
  if (ngpu <= 0 || slots_per_gpu <= 0) return nullptr;
  Sched* s = new Sched();
  s->ngpu = ngpu;
  s->slots_per_gpu = slots_per_gpu;
  s->max_skip = max_skip < 0 ? 0 : max_skip;
  s->load.assign(ngpu, 0);
  s->owners.assign(ngpu, {});
  return s;
}

void csa_sched_destroy(void* h) { delete static_cast<Sched*>(h); }

// Enqueue a job.  Returns 0, or -1 if it can never fit (ngpus > ngpu).
int csa_sched_submit(void* h, int64_t job, int ngpus) {
  Sched& s = *static_cast<Sched*>(h);
  if (ngpus <= 0 || ngpus > s.ngpu) return -1;
  std::lock_guard<std::mutex> lk(s.mu);
  s.queue.push_back({job, ngpus, 0});
  return 0;
}

// Admit the next runnable job.  On success writes its id to *job, its GPU ids to
// gpus_out[0..n) and returns n; returns 0 when nothing can be admitted now.
int csa_sched_next(void* h, int64_t* job, int* gpus_out, int cap) {
  Sched& s = *static_cast<Sched*>(h);
  std::lock_guard<std::mutex> lk(s.mu);
  for (size_t i = 0; i < s.queue.size(); ++i) {
    Pending& p = s.queue[i];
    std::vector<int> g = pick(s, p.ngpus);
    if (!g.empty() && (int)g.size() <= cap) {
      // a job behind a starving head may only pass it max_skip times
      if (i > 0 && s.queue[0].skipped >= s.max_skip) return 0;
      for (size_t j = 0; j < i; ++j) s.queue[j].skipped++;
      place(s, p.job, g);
      *job = p.job;
      for (size_t k = 0; k < g.size(); ++k) gpus_out[k] = g[k];
      s.queue.erase(s.queue.begin() + (long)i);
      return (int)g.size();
    }
  }
  return 0;
}

// Release every slot held by `job` (finished, failed, stopped or paused).
int csa_sched_release(void* h, int64_t job) {
  Sched& s = *static_cast<Sched*>(h);
  std::lock_guard<std::mutex> lk(s.mu);
  int freed = 0;
  for (int g = 0; g < s.ngpu; ++g) {
    auto& o = s.owners[g];
    auto it = std::find(o.begin(), o.end(), job);
    if (it != o.end()) {
      o.erase(it);
      s.load[g]--;
      freed++;
    }
  }
  return freed;
}

// Pin `job` to one slot of GPU `gpu` outside the queue (the API server's resident
// inference models and GPU preprocessing live there: their HBM and CU time is not a
// training job's to take).  Returns 0, or -1 if the GPU id is bad or has no free slot.
// `csa_sched_release(job)` frees it like any job.
int csa_sched_reserve(void* h, int64_t job, int gpu) {
  Sched& s = *static_cast<Sched*>(h);
  std::lock_guard<std::mutex> lk(s.mu);
  if (gpu < 0 || gpu >= s.ngpu || s.load[gpu] >= s.slots_per_gpu) return -1;
  place(s, job, {gpu});
  return 0;
}

// Remove a queued (not yet admitted) job.  Returns 1 if it was queued.
int csa_sched_cancel(void* h, int64_t job) {
  Sched& s = *static_cast<Sched*>(h);
  std::lock_guard<std::mutex> lk(s.mu);
  for (auto it = s.queue.begin(); it != s.queue.end(); ++it)
    if (it->job == job) {
      s.queue.erase(it);
      return 1;
    }
  return 0;
}

int csa_sched_load(void* h, int gpu) {
  Sched& s = *static_cast<Sched*>(h);
  std::lock_guard<std::mutex> lk(s.mu);
  return (gpu >= 0 && gpu < s.ngpu) ? s.load[gpu] : -1;
}

int csa_sched_queued(void* h) {
  Sched& s = *static_cast<Sched*>(h);
  std::lock_guard<std::mutex> lk(s.mu);
  return (int)s.queue.size();
}

}  // extern "C"
