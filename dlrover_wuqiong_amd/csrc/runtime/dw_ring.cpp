// Shared-memory batch ring for data loading across processes of one node.
//
// A fixed number of slots, each large enough for one serialized batch, in one
// POSIX shm segment.  Two modes:
//   * SHARED (mode 0): many producers, many consumers, every batch is taken by
//     exactly one consumer (coworker processes feeding training processes);
//   * BROADCAST (mode 1): one producer, ``nreaders`` consumers that each read
//     EVERY batch in order (rank 0 of a tensor/sequence-parallel group loads,
//     its peers reuse the same batch) -- a slot is recycled when the last
//     reader released it.
// Slot ownership follows the bounded-MPMC sequence scheme: slot i carries a
// sequence word; a producer may fill ticket t when seq == t, a consumer may
// take ticket t when seq == t + 1; tickets are claimed by CAS *after* the slot
// is seen ready, so a timed-out waiter never strands a ticket.  Blocking uses
// a futex on one shared "wake" word (bumped by every state change), in short
// slices, so a killed peer can never leave a waiter blocked forever.
//
// Parity: ATorch ``atorch/data/shm_context.py`` (``ShmDataContext``: coworker
// O1 and model-parallel O2 cases, write/read counters in a state shm) and
// ``shm_dataloader.py``.
#include <fcntl.h>
#include <linux/futex.h>
#include <stdint.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <string>

namespace {

constexpr uint64_t kRingMagic = 0x444d5752494e4731ull;  // "DMWRING1"
constexpr int kMaxReaders = 64;
constexpr uint64_t kHdr = 8192;

struct RingHeader {
  uint64_t magic;
  uint32_t nslots, nreaders, mode, nproducers;
  uint64_t slot_bytes, total;
  std::atomic<uint64_t> write_ticket;
  std::atomic<uint64_t> read_ticket;
  std::atomic<uint32_t> stop;
  std::atomic<uint32_t> wake;
  std::atomic<uint32_t> epoch;
  std::atomic<uint32_t> producers_done;
  std::atomic<uint64_t> cursor[kMaxReaders];
  std::atomic<uint32_t> ended[kMaxReaders];  // epoch + 1 once reader r saw the end of epoch
};
static_assert(sizeof(RingHeader) <= 4096, "ring header too big");

struct SlotHeader {
  std::atomic<uint64_t> seq;
  std::atomic<uint32_t> nread;
  uint32_t pad;
  uint64_t nbytes;
  uint64_t pad2[5];
};
static_assert(sizeof(SlotHeader) == 64, "slot header must be 64 B");

struct Ring {
  RingHeader* h;
  uint64_t total;
};

SlotHeader* slot_hdr(RingHeader* h, uint64_t i) { return (SlotHeader*)((char*)h + 4096) + i; }

uint64_t payload_off(uint32_t nslots) {
  const uint64_t o = 4096 + (uint64_t)nslots * 64;
  return (o + kHdr - 1) / kHdr * kHdr;
}

std::string shm_name(const char* name) {
  std::string s = name;
  if (s.empty() || s[0] != '/') s = "/" + s;
  return s;
}

void wake_all(RingHeader* h) {
  h->wake.fetch_add(1, std::memory_order_acq_rel);
  syscall(SYS_futex, (uint32_t*)&h->wake, FUTEX_WAKE, INT32_MAX, nullptr, nullptr, 0);
}

double now_s() {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

// Wait until pred() or timeout; returns true if pred() held.
template <typename P>
bool wait_for(RingHeader* h, double timeout, P pred) {
  const double end = now_s() + (timeout < 0 ? 1e12 : timeout);
  while (true) {
    const uint32_t seen = h->wake.load(std::memory_order_acquire);
    if (pred()) return true;
    const double left = end - now_s();
    if (left <= 0) return false;
    const double slice = left < 0.05 ? left : 0.05;
    struct timespec rel;
    rel.tv_sec = (time_t)slice;
    rel.tv_nsec = (long)((slice - (double)rel.tv_sec) * 1e9);
    syscall(SYS_futex, (uint32_t*)&h->wake, FUTEX_WAIT, seen, &rel, nullptr, 0);
  }
}

void init_slots(RingHeader* h) {
  for (uint64_t i = 0; i < h->nslots; ++i) {
    SlotHeader* s = slot_hdr(h, i);
    s->seq.store(i, std::memory_order_relaxed);
    s->nread.store(0, std::memory_order_relaxed);
    s->nbytes = 0;
  }
  h->write_ticket.store(0);
  h->read_ticket.store(0);
  for (int r = 0; r < kMaxReaders; ++r) h->cursor[r].store(0);
  h->stop.store(0);
  h->producers_done.store(0);
}

}  // namespace

extern "C" {

void* dw_ring_open(const char* name, int create, uint32_t nslots, uint64_t slot_bytes, uint32_t nreaders,
                   uint32_t mode, uint32_t nproducers, double timeout) {
  const std::string nm = shm_name(name);
  if (create) {
    if (nslots == 0 || nreaders == 0 || nreaders > kMaxReaders) return nullptr;
    slot_bytes = (slot_bytes + kHdr - 1) / kHdr * kHdr;
    const uint64_t total = payload_off(nslots) + (uint64_t)nslots * slot_bytes;
    shm_unlink(nm.c_str());
    int fd = shm_open(nm.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd < 0) return nullptr;
    if (ftruncate(fd, (off_t)total) != 0) {
      close(fd);
      shm_unlink(nm.c_str());
      return nullptr;
    }
    void* p = mmap(nullptr, total, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) return nullptr;
    RingHeader* h = (RingHeader*)p;
    h->nslots = nslots;
    h->nreaders = nreaders;
    h->mode = mode;
    h->nproducers = nproducers ? nproducers : 1;
    h->slot_bytes = slot_bytes;
    h->total = total;
    h->wake.store(0);
    h->epoch.store(0);
    for (int r = 0; r < kMaxReaders; ++r) h->ended[r].store(0);
    init_slots(h);
    std::atomic_thread_fence(std::memory_order_release);
    ((std::atomic<uint64_t>*)&h->magic)->store(kRingMagic, std::memory_order_release);
    return new Ring{h, total};
  }
  // attach: wait for the creator
  const double end = now_s() + (timeout < 0 ? 1e12 : timeout);
  while (true) {
    int fd = shm_open(nm.c_str(), O_RDWR, 0600);
    if (fd >= 0) {
      struct stat st;
      if (fstat(fd, &st) == 0 && st.st_size >= 4096) {
        void* p = mmap(nullptr, st.st_size, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        close(fd);
        if (p == MAP_FAILED) return nullptr;
        RingHeader* h = (RingHeader*)p;
        if (((std::atomic<uint64_t>*)&h->magic)->load(std::memory_order_acquire) == kRingMagic &&
            h->total == (uint64_t)st.st_size)
          return new Ring{h, (uint64_t)st.st_size};
        munmap(p, st.st_size);
      } else {
        close(fd);
      }
    }
    if (now_s() > end) return nullptr;
    usleep(2000);
  }
}

int dw_ring_close(void* r) {
  Ring* R = (Ring*)r;
  if (!R) return -1;
  munmap(R->h, R->total);
  delete R;
  return 0;
}

uint64_t dw_ring_slot_bytes(void* r) { return ((Ring*)r)->h->slot_bytes; }
uint32_t dw_ring_nslots(void* r) { return ((Ring*)r)->h->nslots; }
uint32_t dw_ring_epoch(void* r) { return ((Ring*)r)->h->epoch.load(); }
void* dw_ring_base(void* r) { return ((Ring*)r)->h; }
uint64_t dw_ring_total(void* r) { return ((Ring*)r)->total; }

void* dw_ring_slot(void* r, int64_t ticket) {
  RingHeader* h = ((Ring*)r)->h;
  return (char*)h + payload_off(h->nslots) + (uint64_t)(ticket % h->nslots) * h->slot_bytes;
}

// -> ticket >= 0, -1 timeout, -3 stopped
int64_t dw_ring_write_acquire(void* r, double timeout) {
  RingHeader* h = ((Ring*)r)->h;
  int64_t got = -1;
  bool ok = wait_for(h, timeout, [&] {
    if (h->stop.load(std::memory_order_acquire)) {
      got = -3;
      return true;
    }
    for (;;) {  // a lost CAS means another producer won: retry at once
      uint64_t t = h->write_ticket.load(std::memory_order_acquire);
      SlotHeader* s = slot_hdr(h, t % h->nslots);
      if (s->seq.load(std::memory_order_acquire) != t) return false;
      if (h->write_ticket.compare_exchange_strong(t, t + 1)) {
        got = (int64_t)t;
        return true;
      }
    }
  });
  return ok ? got : -1;
}

int dw_ring_write_commit(void* r, int64_t ticket, uint64_t nbytes) {
  RingHeader* h = ((Ring*)r)->h;
  SlotHeader* s = slot_hdr(h, (uint64_t)ticket % h->nslots);
  s->nbytes = nbytes;
  s->seq.store((uint64_t)ticket + 1, std::memory_order_release);
  wake_all(h);
  return 0;
}

// -> ticket >= 0, -1 timeout, -2 end of data (stopped and drained)
int64_t dw_ring_read_acquire(void* r, int reader, double timeout, uint64_t* nbytes) {
  RingHeader* h = ((Ring*)r)->h;
  int64_t got = -1;
  bool ok = wait_for(h, timeout, [&] {
    for (;;) {
      uint64_t t = h->mode == 1 ? h->cursor[reader].load(std::memory_order_acquire)
                                : h->read_ticket.load(std::memory_order_acquire);
      SlotHeader* s = slot_hdr(h, t % h->nslots);
      if (s->seq.load(std::memory_order_acquire) == t + 1) {
        if (h->mode == 1 || h->read_ticket.compare_exchange_strong(t, t + 1)) {
          got = (int64_t)t;
          if (nbytes) *nbytes = s->nbytes;
          return true;
        }
        continue;  // another consumer took it: try the next ticket
      }
      // stopped and nothing left for this reader
      if (h->stop.load(std::memory_order_acquire) && h->write_ticket.load() <= t) {
        got = -2;
        if (reader >= 0 && reader < kMaxReaders) h->ended[reader].store(h->epoch.load() + 1);
        wake_all(h);  // a producer may wait for this in next_epoch
        return true;
      }
      return false;
    }
  });
  return ok ? got : -1;
}

int dw_ring_read_release(void* r, int reader, int64_t ticket) {
  RingHeader* h = ((Ring*)r)->h;
  SlotHeader* s = slot_hdr(h, (uint64_t)ticket % h->nslots);
  if (h->mode == 1) {
    h->cursor[reader].store((uint64_t)ticket + 1, std::memory_order_release);
    if (s->nread.fetch_add(1) + 1 == h->nreaders) {
      s->nread.store(0);
      s->seq.store((uint64_t)ticket + h->nslots, std::memory_order_release);
    }
  } else {
    s->seq.store((uint64_t)ticket + h->nslots, std::memory_order_release);
  }
  wake_all(h);
  return 0;
}

// Producer: no more batches this epoch from this producer; the epoch ends
// when all ``nproducers`` producers said so.
int dw_ring_stop(void* r) {
  RingHeader* h = ((Ring*)r)->h;
  if (h->producers_done.fetch_add(1) + 1 >= h->nproducers) h->stop.store(1, std::memory_order_release);
  wake_all(h);
  return 0;
}

// Abort: wake everyone, end the epoch regardless of the other producers.
int dw_ring_abort(void* r) {
  RingHeader* h = ((Ring*)r)->h;
  h->stop.store(1, std::memory_order_release);
  wake_all(h);
  return 0;
}

// Producer: wait until every reader drained the stopped epoch, then start a
// new one (tickets/slots re-initialised, epoch + 1).  0 ok, -1 timeout.
int dw_ring_next_epoch(void* r, double timeout) {
  RingHeader* h = ((Ring*)r)->h;
  // every reader must have OBSERVED the end of the current epoch (not just
  // consumed its batches), or it could miss the boundary and run on into the
  // next epoch's data
  const uint32_t e1 = h->epoch.load() + 1;
  bool ok = wait_for(h, timeout, [&] {
    for (uint32_t i = 0; i < h->nreaders; ++i)
      if (h->ended[i].load() < e1) return false;
    return true;
  });
  if (!ok) return -1;
  init_slots(h);
  h->epoch.fetch_add(1, std::memory_order_acq_rel);
  wake_all(h);
  return 0;
}

// Reader: wait for the producer to open epoch ``e``.  0 ok, -1 timeout.
int dw_ring_wait_epoch(void* r, uint32_t e, double timeout) {
  RingHeader* h = ((Ring*)r)->h;
  return wait_for(h, timeout, [&] { return h->epoch.load(std::memory_order_acquire) >= e; }) ? 0 : -1;
}

}  // extern "C"
