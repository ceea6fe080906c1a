// dw_runtime: node-local native runtime for dlrover_wuqiong_amd.
//
// What lives here (all host-side, no GPU dependency so it also serves CPU/gloo
// jobs and the CPU test-suite):
//   * POSIX shared-memory segments that survive a worker crash (the flash
//     checkpoint buffer lives in one), with parallel pre-faulting so the first
//     checkpoint does not pay page-fault cost inside the training loop.
//   * Process-shared, *robust* primitives living in small named shm control
//     blocks: a lock (pthread robust mutex: a worker that dies while holding it
//     does not wedge the agent), a bounded message queue (mutex + 2 condvars,
//     variable-size messages in a ring), and a versioned blob "dict".
//     The reference implements SharedLock/SharedQueue/SharedDict as Python
//     socket servers with pickle framing (reference
//     dlrover/python/common/multi_process.py:162-534); here they are lock-free
//     of any server thread: every process maps the control block directly.
//   * Parallel file IO used by the asynchronous persister: pwrite/pread of a
//     large buffer with N threads, optional fsync, and a parallel memcpy.
//
// C ABI only (loaded through ctypes) so it has no Python/PyTorch ABI coupling.

#include <errno.h>
#include <stdio.h>
#include <fcntl.h>
#include <pthread.h>
#include <signal.h>
#include <linux/futex.h>
#include <sys/syscall.h>
#include <climits>
#include <stdint.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <string>
#include <thread>
#include <vector>

#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23
#endif

extern "C" {

// ---------------------------------------------------------------------------
// Error reporting
// ---------------------------------------------------------------------------
static thread_local char g_err[512];
static void set_err(const char* what) {
  snprintf(g_err, sizeof(g_err), "%s: %s", what, strerror(errno));
}
const char* dw_last_error() { return g_err; }

static std::string shm_path_name(const char* name) {
  std::string n(name);
  if (n.empty() || n[0] != '/') n = "/" + n;
  return n;
}

// ---------------------------------------------------------------------------
// Shared memory segments
// ---------------------------------------------------------------------------
// Create (or re-create with a different size) a named segment and map it.
// Returns the mapped address or nullptr.
void* dw_shm_create(const char* name, uint64_t size, int exclusive) {
  std::string n = shm_path_name(name);
  int flags = O_CREAT | O_RDWR | (exclusive ? O_EXCL : 0);
  int fd = shm_open(n.c_str(), flags, 0600);
  if (fd < 0) { set_err("shm_open(create)"); return nullptr; }
  struct stat st;
  if (fstat(fd, &st) != 0) { set_err("fstat"); close(fd); return nullptr; }
  if ((uint64_t)st.st_size != size) {
    if (ftruncate(fd, (off_t)size) != 0) { set_err("ftruncate"); close(fd); return nullptr; }
  }
  void* p = mmap(nullptr, size, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) { set_err("mmap"); return nullptr; }
  return p;
}

// Open an existing segment; *size receives its length. nullptr if absent.
void* dw_shm_open(const char* name, uint64_t* size) {
  std::string n = shm_path_name(name);
  int fd = shm_open(n.c_str(), O_RDWR, 0600);
  if (fd < 0) { set_err("shm_open"); return nullptr; }
  struct stat st;
  if (fstat(fd, &st) != 0) { set_err("fstat"); close(fd); return nullptr; }
  *size = (uint64_t)st.st_size;
  if (st.st_size == 0) { close(fd); return nullptr; }
  void* p = mmap(nullptr, (size_t)st.st_size, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) { set_err("mmap"); return nullptr; }
  return p;
}

int dw_shm_exists(const char* name) {
  std::string n = "/dev/shm" + shm_path_name(name);
  struct stat st;
  return stat(n.c_str(), &st) == 0 ? 1 : 0;
}

int64_t dw_shm_size(const char* name) {
  std::string n = "/dev/shm" + shm_path_name(name);
  struct stat st;
  if (stat(n.c_str(), &st) != 0) return -1;
  return (int64_t)st.st_size;
}

int dw_shm_close(void* p, uint64_t size) { return munmap(p, size); }

int dw_shm_unlink(const char* name) {
  std::string n = shm_path_name(name);
  int r = shm_unlink(n.c_str());
  if (r != 0 && errno == ENOENT) return 0;
  return r;
}

// Touch every page of [p, p+size) with nthreads so the kernel allocates and
// zeroes them now rather than inside a later (timed) copy.
int dw_prefault(void* p, uint64_t size, int nthreads) {
  if (size == 0) return 0;
  // one kernel-side populate is the fastest on tmpfs (parallel populates of
  // one shmem object contend); touch pages from threads only without it
  if (madvise(p, size, MADV_POPULATE_WRITE) == 0) return 0;
  nthreads = std::max(1, nthreads);
  const uint64_t page = 4096;
  uint64_t per = ((size / nthreads) + page - 1) / page * page;
  std::vector<std::thread> ts;
  for (int t = 0; t < nthreads; ++t) {
    uint64_t b = t * per, e = std::min(size, b + per);
    if (b >= e) break;
    ts.emplace_back([=]() {
      char* base = (char*)p;
      if (madvise(base + b, e - b, MADV_POPULATE_WRITE) == 0) return;
      for (uint64_t o = b; o < e; o += page) {
        volatile char* c = base + o;
        *c = *c;
      }
    });
  }
  for (auto& t : ts) t.join();
  return 0;
}

// ---------------------------------------------------------------------------
// Parallel memcpy / file IO (persist path)
// ---------------------------------------------------------------------------
int dw_memcpy_parallel(void* dst, const void* src, uint64_t n, int nthreads) {
  nthreads = std::max(1, nthreads);
  if (n < (8ull << 20) || nthreads == 1) { memcpy(dst, src, n); return 0; }
  uint64_t per = (n + nthreads - 1) / nthreads;
  per = (per + 4095) / 4096 * 4096;
  std::vector<std::thread> ts;
  for (int t = 0; t < nthreads; ++t) {
    uint64_t b = t * per, e = std::min(n, b + per);
    if (b >= e) break;
    ts.emplace_back([=]() { memcpy((char*)dst + b, (const char*)src + b, e - b); });
  }
  for (auto& t : ts) t.join();
  return 0;
}

// Record the calling worker thread's errno in the shared slot (first failure
// wins; a zero errno still marks failure as EIO).  errno is thread-local, so
// the joining thread must read the workers' value from here.
static void keep_errno(std::atomic<int>& slot) {
  int expect = 0;
  slot.compare_exchange_strong(expect, errno ? errno : EIO);
}

static int pwrite_all(int fd, const char* buf, uint64_t n, uint64_t off) {
  while (n > 0) {
    size_t chunk = (size_t)std::min<uint64_t>(n, 1ull << 30);
    ssize_t w = pwrite(fd, buf, chunk, (off_t)off);
    if (w < 0) { if (errno == EINTR) continue; return -1; }
    buf += w; n -= (uint64_t)w; off += (uint64_t)w;
  }
  return 0;
}

static int pread_all(int fd, char* buf, uint64_t n, uint64_t off) {
  while (n > 0) {
    size_t chunk = (size_t)std::min<uint64_t>(n, 1ull << 30);
    ssize_t r = pread(fd, buf, chunk, (off_t)off);
    if (r < 0) { if (errno == EINTR) continue; return -1; }
    if (r == 0) { errno = EIO; return -1; }
    buf += r; n -= (uint64_t)r; off += (uint64_t)r;
  }
  return 0;
}

// O_DIRECT body of dw_write_file: [0, body) of buf at file_off, 8 MiB work
// items handed out dynamically.  Returns 0, or the errno of the first failure.
static int write_direct_body(int dfd, const char* buf, uint64_t body, uint64_t file_off, int nthreads) {
  const uint64_t item = 8ull << 20;
  std::atomic<uint64_t> next{0};
  std::atomic<int> failed{0};
  int nt = (int)std::min<uint64_t>((uint64_t)std::max(1, nthreads), (body + item - 1) / item);
  std::vector<std::thread> ts;
  for (int t = 0; t < nt; ++t) {
    ts.emplace_back([&]() {
      for (;;) {
        uint64_t b = next.fetch_add(item);
        if (b >= body || failed.load()) break;
        uint64_t e = std::min(body, b + item);
        if (pwrite_all(dfd, buf + b, e - b, file_off + b) != 0) { keep_errno(failed); break; }
      }
    });
  }
  for (auto& t : ts) t.join();
  return failed.load();
}

// Write buf[0:n] at file offset `file_off` of `path` with nthreads concurrent
// pwrite streams. mode: bit0 = truncate/create, bit1 = fsync at the end,
// bit2 = O_DIRECT for the 4 KiB-aligned body when buf and file_off are
// aligned (no page-cache copy and no single-threaded write-back: the
// persister's large records stream at the device's rate; the tail and a
// file system that refuses O_DIRECT take the buffered path).
int dw_write_file(const char* path, const void* buf, uint64_t n, uint64_t file_off,
                  int nthreads, int mode) {
  int flags = O_WRONLY | O_CREAT | ((mode & 1) ? O_TRUNC : 0);
  int fd = open(path, flags, 0644);
  if (fd < 0) { set_err("open(write)"); return -1; }
  nthreads = std::max(1, nthreads);
  const uint64_t A = 4096;
  if ((mode & 4) && n >= (16ull << 20) && ((uintptr_t)buf % A) == 0 && (file_off % A) == 0) {
    int dfd = open(path, O_WRONLY | O_DIRECT);
    if (dfd >= 0) {
      const uint64_t body = n / A * A;
      const int e = write_direct_body(dfd, (const char*)buf, body, file_off, nthreads);
      close(dfd);
      if (e == 0) {
        buf = (const char*)buf + body;
        file_off += body;
        n -= body;
      }  // any failure of the direct path (EINVAL: refused mid-way, or a file
         // system that accepts the flag but fails the writes): everything
         // again through the buffered path, whose errors are the ones reported
    }
  }
  std::atomic<int> failed{0};  // errno of the first failing worker (errno is per thread)
  if (n < (16ull << 20)) nthreads = 1;
  uint64_t per = (n + nthreads - 1) / nthreads;
  per = (per + 4095) / 4096 * 4096;
  std::vector<std::thread> ts;
  for (int t = 0; t < nthreads; ++t) {
    uint64_t b = t * per, e = std::min(n, b + per);
    if (b >= e) break;
    ts.emplace_back([&, b, e]() {
      if (pwrite_all(fd, (const char*)buf + b, e - b, file_off + b) != 0) keep_errno(failed);
    });
  }
  for (auto& t : ts) t.join();
  if (failed) { errno = failed.load(); set_err("pwrite"); close(fd); return -1; }
  if ((mode & 2) && fsync(fd) != 0) { set_err("fsync"); close(fd); return -1; }
  close(fd);
  return 0;
}

int dw_read_file(const char* path, void* buf, uint64_t n, uint64_t file_off, int nthreads) {
  int fd = open(path, O_RDONLY);
  if (fd < 0) { set_err("open(read)"); return -1; }
  nthreads = std::max(1, nthreads);
  if (n < (16ull << 20)) nthreads = 1;
  std::atomic<int> failed{0};
  uint64_t per = (n + nthreads - 1) / nthreads;
  per = (per + 4095) / 4096 * 4096;
  std::vector<std::thread> ts;
  for (int t = 0; t < nthreads; ++t) {
    uint64_t b = t * per, e = std::min(n, b + per);
    if (b >= e) break;
    ts.emplace_back([&, b, e]() {
      if (pread_all(fd, (char*)buf + b, e - b, file_off + b) != 0) keep_errno(failed);
    });
  }
  for (auto& t : ts) t.join();
  close(fd);
  if (failed) { errno = failed.load(); set_err("pread"); return -1; }
  return 0;
}

// Cold read of a persisted checkpoint range into host memory.
// flags bit0: O_DIRECT (bypass the page cache: what a restore after a node
// replacement sees); the 4 KiB-aligned body is read with nthreads concurrent
// O_DIRECT streams and the unaligned tail (or everything, when the file system
// refuses O_DIRECT or buf/off are unaligned) through the page cache.
// flags bit1: posix_fadvise(DONTNEED) over the range first (drops clean cached
// pages: a buffered read then also comes from the device).
// Returns 1 if O_DIRECT was used for the body, 0 if buffered, -1 on error.
int dw_read_file_direct(const char* path, void* buf, uint64_t n, uint64_t file_off, int nthreads, int flags) {
  const uint64_t A = 4096;
  if (flags & 2) {
    int fd0 = open(path, O_RDONLY);
    if (fd0 >= 0) { posix_fadvise(fd0, (off_t)file_off, (off_t)n, POSIX_FADV_DONTNEED); close(fd0); }
  }
  uint64_t body = 0;
  int dfd = -1;
  if ((flags & 1) && ((uintptr_t)buf % A) == 0 && (file_off % A) == 0) {
    dfd = open(path, O_RDONLY | O_DIRECT);
    if (dfd >= 0) body = n / A * A;
  }
  nthreads = std::max(1, nthreads);
  std::atomic<int> failed{0};
  if (body > 0) {
    // 8 MiB-granular work items handed out dynamically: O_DIRECT streams keep
    // the device queue deep without one slow thread holding the tail
    const uint64_t item = 8ull << 20;
    std::atomic<uint64_t> next{0};
    int nt = (int)std::min<uint64_t>((uint64_t)nthreads, (body + item - 1) / item);
    std::vector<std::thread> ts;
    for (int t = 0; t < nt; ++t) {
      ts.emplace_back([&]() {
        for (;;) {
          uint64_t b = next.fetch_add(item);
          if (b >= body || failed.load()) break;
          uint64_t e = std::min(body, b + item);
          char* dst = (char*)buf + b;
          uint64_t m = e - b, off = file_off + b;
          while (m > 0) {
            ssize_t r = pread(dfd, dst, (size_t)m, (off_t)off);
            if (r < 0) { if (errno == EINTR) continue; keep_errno(failed); break; }
            if (r == 0) { errno = EIO; keep_errno(failed); break; }
            dst += r; m -= (uint64_t)r; off += (uint64_t)r;
            if (m % A) break;  // short read at EOF: the buffered tail path finishes it
          }
        }
      });
    }
    for (auto& t : ts) t.join();
    close(dfd);
    if (failed) {
      const int e = failed.load();
      if (e == EINVAL) { body = 0; failed = 0; }  // O_DIRECT refused mid-way: redo buffered
      else { errno = e; set_err("pread(O_DIRECT)"); return -1; }
    }
  } else if (dfd >= 0) {
    close(dfd);
  }
  if (body < n) {
    if (dw_read_file(path, (char*)buf + body, n - body, file_off + body, nthreads) != 0) return -1;
  }
  return body > 0 ? 1 : 0;
}

// CRC32C (Castagnoli), slicing-by-1 table; used to verify persisted shards.
static uint32_t g_crc_table[256];
static std::atomic<int> g_crc_init{0};
static void crc_init() {
  if (g_crc_init.load()) return;
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (0x82F63B78u ^ (c >> 1)) : (c >> 1);
    g_crc_table[i] = c;
  }
  g_crc_init = 1;
}
uint32_t dw_crc32c(const void* data, uint64_t n, uint32_t seed) {
  crc_init();
  const uint8_t* p = (const uint8_t*)data;
  uint32_t c = ~seed;
#if defined(__SSE4_2__)
  while (n >= 8) { c = (uint32_t)__builtin_ia32_crc32di(c, *(const uint64_t*)p); p += 8; n -= 8; }
  while (n--) c = __builtin_ia32_crc32qi(c, *p++);
#else
  while (n--) c = g_crc_table[(c ^ *p++) & 0xFF] ^ (c >> 8);
#endif
  return ~c;
}

// ---------------------------------------------------------------------------
// Control blocks: robust lock, queue, blob dict
// ---------------------------------------------------------------------------
// Waiting uses futexes on sequence words instead of process-shared condition
// variables: a glibc condvar signal can block forever when one of its waiters
// was SIGKILLed (it waits for the dead waiter to leave its group), and killed
// agents/workers are exactly what this runtime must survive.  FUTEX_WAKE never
// blocks, and a dead waiter simply never consumes its wake-up.
static const uint64_t kMagic = 0x44574d4443544c32ull;  // "DWMDCTL2"

struct CtlHeader {
  std::atomic<uint64_t> magic;
  pthread_mutex_t mu;
  std::atomic<uint32_t> seq_not_empty;
  std::atomic<uint32_t> seq_not_full;
  uint32_t kind;       // 1 lock, 2 queue, 3 dict
  uint32_t pad0;
  uint64_t capacity;   // queue: max messages
  uint64_t data_size;  // bytes of payload area
  // queue ring state
  uint64_t head;       // byte offset of the oldest message
  uint64_t tail;       // byte offset where the next message goes
  uint64_t count;      // messages in the queue
  uint64_t used;       // bytes used in ring (incl. 8-byte length prefixes)
  // dict state
  uint64_t version;
  uint64_t blob_len;
  // lock state
  int32_t held;
  int32_t holder_pid;
};

static uint64_t ctl_total(uint64_t data_size) {
  return (sizeof(CtlHeader) + 63) / 64 * 64 + data_size;
}
static char* ctl_data(CtlHeader* h) { return (char*)h + (sizeof(CtlHeader) + 63) / 64 * 64; }

static int robust_lock(CtlHeader* h) {
  int r = pthread_mutex_lock(&h->mu);
  if (r == EOWNERDEAD) { pthread_mutex_consistent(&h->mu); r = 0; }
  return r;
}

static void seq_notify(std::atomic<uint32_t>* w) {
  w->fetch_add(1, std::memory_order_release);
  syscall(SYS_futex, (uint32_t*)w, FUTEX_WAKE, INT32_MAX, nullptr, nullptr, 0);
}

// Called with h->mu held; releases it, sleeps until *w changes (or at most
// `slice_s`), re-acquires it.  Spurious wake-ups are fine: callers re-check.
static int seq_wait_unlocked(CtlHeader* h, std::atomic<uint32_t>* w, double slice_s) {
  uint32_t seen = w->load(std::memory_order_acquire);
  pthread_mutex_unlock(&h->mu);
  struct timespec rel;
  rel.tv_sec = (time_t)slice_s;
  rel.tv_nsec = (long)((slice_s - (double)rel.tv_sec) * 1e9);
  syscall(SYS_futex, (uint32_t*)w, FUTEX_WAIT, seen, &rel, nullptr, 0);
  return robust_lock(h);
}

static double secs_left(const struct timespec* dl) {
  struct timespec now;
  clock_gettime(CLOCK_MONOTONIC, &now);
  return (double)(dl->tv_sec - now.tv_sec) + 1e-9 * (double)(dl->tv_nsec - now.tv_nsec);
}

static void abs_deadline(struct timespec* ts, double timeout_s) {
  clock_gettime(CLOCK_MONOTONIC, ts);
  long sec = (long)timeout_s;
  long nsec = (long)((timeout_s - (double)sec) * 1e9);
  ts->tv_sec += sec;
  ts->tv_nsec += nsec;
  if (ts->tv_nsec >= 1000000000L) { ts->tv_sec += 1; ts->tv_nsec -= 1000000000L; }
}

// Returns the mapped control block. create=1 initialises it (idempotent if a
// live block with the same kind already exists).
void* dw_ctl_open(const char* name, int create, uint32_t kind, uint64_t capacity,
                  uint64_t data_size) {
  std::string n = shm_path_name(name);
  uint64_t total = ctl_total(data_size);
  if (create) {
    int fd = shm_open(n.c_str(), O_CREAT | O_RDWR | O_EXCL, 0600);
    bool fresh = fd >= 0;
    if (!fresh) {
      // Exists already: attach (e.g. agent restarted while workers alive).
      uint64_t sz = 0;
      void* p = nullptr;
      // The creator may still be initialising the block: give it up to 2 s.
      for (int spin = 0; spin < 200; ++spin) {
        p = dw_shm_open(name, &sz);
        if (p && sz >= sizeof(CtlHeader) && ((CtlHeader*)p)->magic.load() == kMagic) break;
        if (p) { munmap(p, sz); p = nullptr; }
        usleep(10000);
      }
      if (p && sz >= sizeof(CtlHeader)) {
        CtlHeader* h = (CtlHeader*)p;
        if (h->magic.load() == kMagic && h->kind == kind && sz == total) return p;
        munmap(p, sz);
      }
      shm_unlink(n.c_str());
      fd = shm_open(n.c_str(), O_CREAT | O_RDWR | O_EXCL, 0600);
      if (fd < 0) { set_err("shm_open(ctl)"); return nullptr; }
    }
    if (ftruncate(fd, (off_t)total) != 0) { set_err("ftruncate(ctl)"); close(fd); return nullptr; }
    void* p = mmap(nullptr, total, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) { set_err("mmap(ctl)"); return nullptr; }
    CtlHeader* h = (CtlHeader*)p;
    memset((void*)h, 0, sizeof(CtlHeader));
    pthread_mutexattr_t ma;
    pthread_mutexattr_init(&ma);
    pthread_mutexattr_setpshared(&ma, PTHREAD_PROCESS_SHARED);
    pthread_mutexattr_setrobust(&ma, PTHREAD_MUTEX_ROBUST);
    pthread_mutex_init(&h->mu, &ma);
    pthread_mutexattr_destroy(&ma);
    h->seq_not_empty.store(0);
    h->seq_not_full.store(0);
    h->kind = kind;
    h->capacity = capacity;
    h->data_size = data_size;
    h->magic.store(kMagic);
    return p;
  }
  uint64_t sz = 0;
  void* p = dw_shm_open(name, &sz);
  if (!p) return nullptr;
  CtlHeader* h = (CtlHeader*)p;
  if (sz < sizeof(CtlHeader) || h->magic.load() != kMagic || h->kind != kind) {
    munmap(p, sz);
    errno = EINVAL;
    set_err("ctl block not initialised");
    return nullptr;
  }
  return p;
}

int dw_ctl_close(void* p) {
  CtlHeader* h = (CtlHeader*)p;
  return munmap(p, ctl_total(h->data_size));
}

// ---- lock -----------------------------------------------------------------
// The "held" flag is separate from the pthread mutex so that acquire/release
// may happen from different threads (the reference's SharedLock semantics).
// timeout < 0 blocks forever; returns 1 acquired, 0 not acquired.
// A lock holder that no longer runs: gone (ESRCH) or a zombie / dying task
// whose exit has not been reaped yet.  A SIGKILLed worker with tens of GB of
// mappings stays a zombie for ~1 s while its address space is torn down; its
// locks must be reclaimable at once, or the restarted worker's first saves
// see every slot "held".
static bool pid_gone(pid_t pid) {
  if (kill(pid, 0) != 0) return errno == ESRCH;
  char path[64];
  snprintf(path, sizeof(path), "/proc/%d/stat", (int)pid);
  int fd = open(path, O_RDONLY);
  if (fd < 0) return false;
  char buf[512];
  ssize_t n = read(fd, buf, sizeof(buf) - 1);
  close(fd);
  if (n <= 0) return false;
  buf[n] = 0;
  const char* rp = strrchr(buf, ')');  // comm may contain spaces / parens
  if (!rp || rp[1] != ' ') return false;
  char st = rp[2];
  return st == 'Z' || st == 'X' || st == 'x';
}

int dw_lock_acquire(void* p, int blocking, double timeout) {
  CtlHeader* h = (CtlHeader*)p;
  if (robust_lock(h) != 0) return 0;
  if (h->held && h->holder_pid > 0 && pid_gone(h->holder_pid)) {
    h->held = 0;  // holder died without releasing
  }
  if (!blocking) {
    int ok = !h->held;
    if (ok) { h->held = 1; h->holder_pid = getpid(); }
    pthread_mutex_unlock(&h->mu);
    return ok;
  }
  struct timespec dl;
  if (timeout >= 0) abs_deadline(&dl, timeout);
  while (h->held) {
    // wake at least every 100 ms to detect dead holders
    double slice = 0.1;
    if (timeout >= 0) {
      double left = secs_left(&dl);
      if (left <= 0) { pthread_mutex_unlock(&h->mu); return 0; }
      if (left < slice) slice = left;
    }
    if (seq_wait_unlocked(h, &h->seq_not_full, slice) != 0) return 0;
    if (h->held && h->holder_pid > 0 && pid_gone(h->holder_pid)) h->held = 0;
  }
  h->held = 1;
  h->holder_pid = getpid();
  pthread_mutex_unlock(&h->mu);
  return 1;
}

int dw_lock_release(void* p) {
  CtlHeader* h = (CtlHeader*)p;
  if (robust_lock(h) != 0) return -1;
  h->held = 0;
  h->holder_pid = 0;
  pthread_mutex_unlock(&h->mu);
  seq_notify(&h->seq_not_full);
  return 0;
}

int dw_lock_locked(void* p) {
  CtlHeader* h = (CtlHeader*)p;
  if (robust_lock(h) != 0) return 0;
  if (h->held && h->holder_pid > 0 && pid_gone(h->holder_pid)) h->held = 0;
  int r = h->held;
  pthread_mutex_unlock(&h->mu);
  return r;
}

// ---- queue ----------------------------------------------------------------
// Messages are stored contiguously as [u64 len][bytes...] padded to 8 bytes,
// wrapping with a zero-length "skip" marker when a message does not fit the
// tail of the ring.
static uint64_t pad8(uint64_t x) { return (x + 7) & ~7ull; }

// returns 0 ok, 1 timeout/full, -1 error (message too large)
int dw_queue_put(void* p, const void* msg, uint64_t len, int blocking, double timeout) {
  CtlHeader* h = (CtlHeader*)p;
  uint64_t need = 8 + pad8(len);
  if (need + 8 > h->data_size) return -1;
  if (robust_lock(h) != 0) return -1;
  struct timespec dl;
  if (timeout >= 0) abs_deadline(&dl, timeout);
  for (;;) {
    bool has_slot = h->count < h->capacity;
    // space check (conservative: need + possible wrap waste)
    uint64_t tail_room = h->data_size - h->tail;
    uint64_t waste = (tail_room < need) ? tail_room : 0;
    bool has_space = h->used + need + waste <= h->data_size;
    if (has_slot && has_space) {
      char* d = ctl_data(h);
      if (waste) {
        if (tail_room >= 8) *(uint64_t*)(d + h->tail) = ~0ull;  // wrap marker
        h->used += waste;
        h->tail = 0;
      }
      *(uint64_t*)(d + h->tail) = len;
      memcpy(d + h->tail + 8, msg, len);
      h->tail += need;
      if (h->tail >= h->data_size) h->tail = 0;
      h->used += need;
      h->count += 1;
      pthread_mutex_unlock(&h->mu);
      seq_notify(&h->seq_not_empty);
      return 0;
    }
    if (!blocking) { pthread_mutex_unlock(&h->mu); return 1; }
    double slice = 0.1;
    if (timeout >= 0) {
      double left = secs_left(&dl);
      if (left <= 0) { pthread_mutex_unlock(&h->mu); return 1; }
      if (left < slice) slice = left;
    }
    if (seq_wait_unlocked(h, &h->seq_not_full, slice) != 0) return -1;
  }
}

// Pops a message into buf (cap bytes). Returns message length (>=0),
// -1 timeout/empty, -2 buffer too small (message kept; required size in *need).
int64_t dw_queue_get(void* p, void* buf, uint64_t cap, int blocking, double timeout,
                     uint64_t* need_out) {
  CtlHeader* h = (CtlHeader*)p;
  if (robust_lock(h) != 0) return -1;
  struct timespec dl;
  if (timeout >= 0) abs_deadline(&dl, timeout);
  while (h->count == 0) {
    if (!blocking) { pthread_mutex_unlock(&h->mu); return -1; }
    double slice = 0.1;
    if (timeout >= 0) {
      double left = secs_left(&dl);
      if (left <= 0) { pthread_mutex_unlock(&h->mu); return -1; }
      if (left < slice) slice = left;
    }
    if (seq_wait_unlocked(h, &h->seq_not_empty, slice) != 0) return -1;
  }
  char* d = ctl_data(h);
  uint64_t tail_room = h->data_size - h->head;
  if (tail_room < 8 || *(uint64_t*)(d + h->head) == ~0ull) {
    h->used -= tail_room;
    h->head = 0;
  }
  uint64_t len = *(uint64_t*)(d + h->head);
  if (len > cap) {
    if (need_out) *need_out = len;
    pthread_mutex_unlock(&h->mu);
    return -2;
  }
  memcpy(buf, d + h->head + 8, len);
  uint64_t sz = 8 + pad8(len);
  h->head += sz;
  if (h->head >= h->data_size) h->head = 0;
  h->used -= sz;
  h->count -= 1;
  if (h->count == 0) { h->head = h->tail = 0; h->used = 0; }
  pthread_mutex_unlock(&h->mu);
  seq_notify(&h->seq_not_full);
  return (int64_t)len;
}

int64_t dw_queue_size(void* p) {
  CtlHeader* h = (CtlHeader*)p;
  if (robust_lock(h) != 0) return -1;
  int64_t c = (int64_t)h->count;
  pthread_mutex_unlock(&h->mu);
  return c;
}

// ---- dict (versioned blob) -----------------------------------------------
int dw_blob_set(void* p, const void* data, uint64_t len) {
  CtlHeader* h = (CtlHeader*)p;
  if (len > h->data_size) return -1;
  if (robust_lock(h) != 0) return -1;
  memcpy(ctl_data(h), data, len);
  h->blob_len = len;
  h->version += 1;
  pthread_mutex_unlock(&h->mu);
  seq_notify(&h->seq_not_empty);
  return 0;
}

// Returns length, or -2 if cap too small (*need set), or -1 on error.
int64_t dw_blob_get(void* p, void* buf, uint64_t cap, uint64_t* need_out, uint64_t* version) {
  CtlHeader* h = (CtlHeader*)p;
  if (robust_lock(h) != 0) return -1;
  uint64_t len = h->blob_len;
  if (version) *version = h->version;
  if (len > cap) {
    if (need_out) *need_out = len;
    pthread_mutex_unlock(&h->mu);
    return -2;
  }
  memcpy(buf, ctl_data(h), len);
  pthread_mutex_unlock(&h->mu);
  return (int64_t)len;
}

uint64_t dw_blob_version(void* p) {
  CtlHeader* h = (CtlHeader*)p;
  return __atomic_load_n(&h->version, __ATOMIC_ACQUIRE);
}

int dw_runtime_abi_version() { return 1; }

}  // extern "C"
