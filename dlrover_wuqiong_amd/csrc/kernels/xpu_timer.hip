// xpu_timer: low-overhead device-side timing of GEMMs / collectives and
// device-hang detection, driven by HIP events.
//
// The training thread brackets an op with dw_xt_begin / dw_xt_end, which
// record two pooled hipEvents on the op's stream (two ~1 us hipEventRecord
// calls, no host synchronisation).  A poller thread drains completed records
// (hipEventQuery + hipEventElapsedTime) into per-key statistics: count, sum,
// max, a 1024-sample ring for percentiles, and the op's work (FLOPs or bytes)
// for TFLOP/s and bus bandwidth.  Because the poller sees the event timeline
// it also detects a HANG: the oldest record whose end event has not completed
// for longer than the timeout names the op the device is stuck in (its start
// event completed) or the op the device never reached (start not completed).
//
// Parity: ATorch ``atorch/dev/xpu_timer`` (LD_PRELOAD hook of cuBLAS/NCCL
// launches -> CUDA events -> bvar/prometheus; ``common/manager.cc`` poller).
// Here the interposition happens in Python (torch function mode +
// torch.distributed wrappers, see utils/xpu_timer.py) so no preload library
// is needed, and the event machinery is native HIP.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace {

constexpr int kRing = 1024;

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Record {
  hipEvent_t s = nullptr, e = nullptr;
  int key = -1;
  double work = 0;   // FLOPs or bytes
  double t_enq = 0;  // host time of dw_xt_end
  bool start_seen = false;
  double t_start_seen = 0;
};

struct Stat {
  uint64_t n = 0;
  double sum_us = 0, max_us = 0, work = 0;
  float ring[kRing];
  int ring_n = 0, ring_i = 0;
};

struct Timer {
  std::mutex mu;
  std::vector<std::string> names;
  std::unordered_map<std::string, int> ids;
  std::vector<Stat> stats;
  std::vector<hipEvent_t> pool;
  std::unordered_map<int64_t, Record> open;  // begin recorded, end not yet
  std::vector<Record> pending;               // both recorded, not complete
  int64_t next_token = 1;
  std::thread poller;
  std::atomic<bool> running{false};
  double hang_timeout = 300;
  int poll_ms = 50;
  // hang state
  int hang = 0;
  std::string hang_desc;
  double hang_for = 0;
  uint64_t dropped = 0;
};

Timer& T() {
  static Timer* t = new Timer();  // never destroyed: the poller may outlive static dtors
  return *t;
}

hipEvent_t get_event(Timer& t) {
  if (!t.pool.empty()) {
    hipEvent_t e = t.pool.back();
    t.pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

void add_sample(Stat& st, double us, double work) {
  st.n++;
  st.sum_us += us;
  st.max_us = std::max(st.max_us, us);
  st.work += work;
  st.ring[st.ring_i] = (float)us;
  st.ring_i = (st.ring_i + 1) % kRing;
  st.ring_n = std::min(st.ring_n + 1, kRing);
}

void poll_once(Timer& t) {
  std::vector<Record> work;
  {
    std::lock_guard<std::mutex> g(t.mu);
    work.swap(t.pending);
  }
  std::vector<Record> keep;
  std::vector<std::pair<Record, float>> done;
  const double now = now_s();
  for (auto& r : work) {
    if (hipEventQuery(r.e) == hipSuccess) {
      float ms = 0.f;
      if (hipEventElapsedTime(&ms, r.s, r.e) != hipSuccess) ms = -1.f;
      done.emplace_back(r, ms);
    } else {
      if (!r.start_seen && hipEventQuery(r.s) == hipSuccess) {
        r.start_seen = true;
        r.t_start_seen = now;
      }
      keep.push_back(r);
    }
  }
  std::lock_guard<std::mutex> g(t.mu);
  for (auto& d : done) {
    if (d.second >= 0.f) add_sample(t.stats[d.first.key], d.second * 1000.0, d.first.work);
    t.pool.push_back(d.first.s);
    t.pool.push_back(d.first.e);
  }
  // records added while we polled go after the older ones
  keep.insert(keep.end(), t.pending.begin(), t.pending.end());
  t.pending.swap(keep);
  // hang check: oldest unfinished record
  int hang = 0;
  std::string desc;
  double for_s = 0;
  for (auto& r : t.pending) {
    if (r.start_seen && now - r.t_start_seen > t.hang_timeout) {
      hang = 1;
      for_s = now - r.t_start_seen;
      desc = "device stuck in " + t.names[r.key];
      break;
    }
  }
  if (!hang) {
    for (auto& r : t.pending) {
      if (!r.start_seen && now - r.t_enq > t.hang_timeout) {
        hang = 2;
        for_s = now - r.t_enq;
        desc = "device never reached " + t.names[r.key] + " (stuck in earlier work)";
        break;
      }
    }
  }
  t.hang = hang;
  t.hang_desc = desc;
  t.hang_for = for_s;
}

}  // namespace

extern "C" {

int dw_xt_start(double hang_timeout_s, int poll_ms) {
  Timer& t = T();
  t.hang_timeout = hang_timeout_s > 0 ? hang_timeout_s : 300;
  t.poll_ms = poll_ms > 0 ? poll_ms : 50;
  bool expected = false;
  if (!t.running.compare_exchange_strong(expected, true)) return 0;
  t.poller = std::thread([&t] {
    while (t.running.load()) {
      poll_once(t);
      std::this_thread::sleep_for(std::chrono::milliseconds(t.poll_ms));
    }
  });
  return 0;
}

int dw_xt_stop() {
  Timer& t = T();
  bool expected = true;
  if (!t.running.compare_exchange_strong(expected, false)) return 0;
  if (t.poller.joinable()) t.poller.join();
  return 0;
}

// Flush: poll until nothing is pending or timeout (used by tests / snapshots).
int dw_xt_flush(double timeout_s) {
  Timer& t = T();
  const double end = now_s() + timeout_s;
  while (true) {
    poll_once(t);
    {
      std::lock_guard<std::mutex> g(t.mu);
      if (t.pending.empty()) return 0;
    }
    if (now_s() > end) return 1;
    std::this_thread::sleep_for(std::chrono::milliseconds(1));
  }
}

int dw_xt_key(const char* name) {
  Timer& t = T();
  std::lock_guard<std::mutex> g(t.mu);
  auto it = t.ids.find(name);
  if (it != t.ids.end()) return it->second;
  const int id = (int)t.names.size();
  t.names.emplace_back(name);
  t.ids.emplace(name, id);
  t.stats.emplace_back();
  return id;
}

int64_t dw_xt_begin(int key, void* stream) {
  Timer& t = T();
  std::lock_guard<std::mutex> g(t.mu);
  if (key < 0 || key >= (int)t.names.size()) return -1;
  if (t.pending.size() + t.open.size() > 65536) {  // poller not running / device stalled
    t.dropped++;
    return -1;
  }
  Record r;
  r.key = key;
  r.s = get_event(t);
  r.e = get_event(t);
  if (!r.s || !r.e) return -1;
  if (hipEventRecord(r.s, (hipStream_t)stream) != hipSuccess) {
    t.pool.push_back(r.s);
    t.pool.push_back(r.e);
    return -1;
  }
  const int64_t tok = t.next_token++;
  t.open.emplace(tok, r);
  return tok;
}

int dw_xt_end(int64_t token, double work, void* stream) {
  Timer& t = T();
  std::lock_guard<std::mutex> g(t.mu);
  auto it = t.open.find(token);
  if (it == t.open.end()) return -1;
  Record r = it->second;
  t.open.erase(it);
  r.work = work;
  r.t_enq = now_s();
  hipError_t e = hipEventRecord(r.e, (hipStream_t)stream);
  if (e != hipSuccess) {
    t.pool.push_back(r.s);
    t.pool.push_back(r.e);
    return (int)e;
  }
  t.pending.push_back(r);
  return 0;
}

// One line per key: name \t count \t avg_us \t max_us \t p50_us \t p99_us \t work_per_us
// (work/us = MFLOP/s*1e-6... i.e. FLOPs per us = MFLOP/s; callers scale).
int dw_xt_snapshot(char* buf, int cap) {
  Timer& t = T();
  std::string out;
  {
    std::lock_guard<std::mutex> g(t.mu);
    for (size_t i = 0; i < t.names.size(); ++i) {
      const Stat& st = t.stats[i];
      if (st.n == 0) continue;
      std::vector<float> v(st.ring, st.ring + st.ring_n);
      std::sort(v.begin(), v.end());
      auto pct = [&](double p) {
        if (v.empty()) return 0.0;
        size_t k = (size_t)std::min<double>(v.size() - 1, std::floor(p * (v.size() - 1) + 0.5));
        return (double)v[k];
      };
      char line[512];
      snprintf(line, sizeof(line), "%s\t%llu\t%.3f\t%.3f\t%.3f\t%.3f\t%.6e\n", t.names[i].c_str(),
               (unsigned long long)st.n, st.sum_us / st.n, st.max_us, pct(0.5), pct(0.99),
               st.sum_us > 0 ? st.work / st.sum_us : 0.0);
      out += line;
    }
  }
  const int n = (int)std::min<size_t>(out.size(), cap > 0 ? (size_t)cap - 1 : 0);
  if (cap > 0) {
    memcpy(buf, out.data(), n);
    buf[n] = 0;
  }
  return (int)out.size();
}

// Returns 0 (no hang), 1 (stuck inside a timed op), 2 (stuck before one).
int dw_xt_hang(char* buf, int cap, double* seconds) {
  Timer& t = T();
  std::lock_guard<std::mutex> g(t.mu);
  if (seconds) *seconds = t.hang_for;
  if (cap > 0) {
    const int n = (int)std::min<size_t>(t.hang_desc.size(), (size_t)cap - 1);
    memcpy(buf, t.hang_desc.data(), n);
    buf[n] = 0;
  }
  return t.hang;
}

void dw_xt_reset() {
  Timer& t = T();
  std::lock_guard<std::mutex> g(t.mu);
  for (auto& st : t.stats) st = Stat();
  t.dropped = 0;
}

int64_t dw_xt_pending() {
  Timer& t = T();
  std::lock_guard<std::mutex> g(t.mu);
  return (int64_t)(t.pending.size() + t.open.size());
}

}  // extern "C"
