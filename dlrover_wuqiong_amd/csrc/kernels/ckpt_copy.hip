// Flash-checkpoint data movement on the GPU side.
//
//  * dw_multi_copy: ONE launch that copies an arbitrary list of byte ranges
//    (device->device).  Used to (a) snapshot a training state into a staging
//    buffer laid out exactly like the host shared-memory segment, and (b)
//    scatter a restored staging buffer back into the live parameter /
//    optimizer tensors.  The reference copies tensor-by-tensor with
//    `torch.frombuffer(...).copy_(gpu_tensor)` — a synchronous D2H into
//    pageable memory per tensor (reference
//    dlrover/python/elastic_agent/torch/ckpt_saver.py:197-206).  Here the
//    training loop only pays an HBM->HBM copy (~5 TB/s class) and the PCIe
//    transfer runs later on a side stream into pinned shm.
//  * host helpers: pinned registration of the shm segment and async copies on
//    an explicit stream (so the D2H/H2D overlap with training).
#include "dw_common.h"

#include <cstring>

struct CopyDesc {
  const char* src;
  char* dst;
  int64_t nbytes;
};

// Each block walks descriptors in a grid-stride manner over "chunks".
// Descriptors are pre-split on the host into <= chunk_bytes pieces so the work
// per descriptor is bounded and the grid fills all 256 CUs.  U independent
// 16-byte loads in flight per lane; NT: nontemporal (streaming) loads/stores.
template <int U, bool NT>
__global__ void __launch_bounds__(256) multi_copy_kernel(const CopyDesc* __restrict__ descs,
                                                         int64_t n) {
  for (int64_t d = blockIdx.x; d < n; d += gridDim.x) {
    CopyDesc c = descs[d];
    const uintptr_t sa = (uintptr_t)c.src, da = (uintptr_t)c.dst;
    if (((sa ^ da) & 15) == 0 && c.nbytes >= 64) {
      // same misalignment: bytewise head, 16B-vector body, bytewise tail
      const int64_t head = (int64_t)((16 - (sa & 15)) & 15);
      const int64_t nv = (c.nbytes - head) >> 4;
      const int64_t tail0 = head + (nv << 4);
      if ((int64_t)threadIdx.x < head) c.dst[threadIdx.x] = c.src[threadIdx.x];
      for (int64_t i = tail0 + threadIdx.x; i < c.nbytes; i += 256) c.dst[i] = c.src[i];
      const u32x4* s = (const u32x4*)(c.src + head);
      u32x4* t = (u32x4*)(c.dst + head);
      int64_t i = threadIdx.x;
      for (; i + (U - 1) * 256 < nv; i += U * 256) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = NT ? __builtin_nontemporal_load(s + i + u * 256) : s[i + u * 256];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (NT)
            __builtin_nontemporal_store(v[u], t + i + u * 256);
          else
            t[i + u * 256] = v[u];
        }
      }
      for (; i < nv; i += 256) __builtin_nontemporal_store(__builtin_nontemporal_load(s + i), t + i);
    } else if (((sa | da | (uintptr_t)c.nbytes) & 3) == 0) {
      const unsigned int* s = (const unsigned int*)c.src;
      unsigned int* t = (unsigned int*)c.dst;
      int64_t nw = c.nbytes >> 2;
      for (int64_t i = threadIdx.x; i < nw; i += 256) t[i] = s[i];
    } else {
      for (int64_t i = threadIdx.x; i < c.nbytes; i += 256) c.dst[i] = c.src[i];
    }
  }
}

// A/B variants of the snapshot copy (scripts/bench_snapshot_copy.py):
// 0 = U4 nontemporal (default), 1 = U8 nontemporal, 2 = U4 temporal, 3 = U8 temporal.
extern "C" int dw_multi_copy_variant(const void* descs_dev, int64_t n, int variant, int max_blocks, void* stream) {
  if (n <= 0) return 0;
  const int64_t cap = max_blocks > 0 ? max_blocks : 4096;
  const int grid = (int)(n < cap ? n : cap);
  hipStream_t s = (hipStream_t)stream;
  const CopyDesc* d = (const CopyDesc*)descs_dev;
  switch (variant) {
    case 1: hipLaunchKernelGGL((multi_copy_kernel<8, true>), dim3(grid), dim3(256), 0, s, d, n); break;
    case 2: hipLaunchKernelGGL((multi_copy_kernel<4, false>), dim3(grid), dim3(256), 0, s, d, n); break;
    case 3: hipLaunchKernelGGL((multi_copy_kernel<8, false>), dim3(grid), dim3(256), 0, s, d, n); break;
    default: hipLaunchKernelGGL((multi_copy_kernel<4, true>), dim3(grid), dim3(256), 0, s, d, n); break;
  }
  DW_LAUNCH_RET;
}

// max_blocks > 0 bounds the grid: a background snapshot copy that trickles
// through a few CUs beside the training kernels instead of taking the chip.
extern "C" int dw_multi_copy_grid(const void* descs_dev, int64_t n, int max_blocks, void* stream) {
  return dw_multi_copy_variant(descs_dev, n, 0, max_blocks, stream);
}

extern "C" int dw_multi_copy(const void* descs_dev, int64_t n, void* stream) {
  return dw_multi_copy_grid(descs_dev, n, 0, stream);
}

// Fill `n` bytes with a byte value (used to poison buffers in tests).
__global__ void fill_u32_kernel(unsigned int* p, int64_t n, unsigned int v) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    p[i] = v;
}
extern "C" int dw_fill_u32(void* p, int64_t n, unsigned int v, void* stream) {
  hipLaunchKernelGGL(fill_u32_kernel, dim3(dw_grid_for(n, 256)), dim3(256), 0,
                     (hipStream_t)stream, (unsigned int*)p, n, v);
  DW_LAUNCH_RET;
}

// ------------------------------ host helpers -------------------------------
extern "C" int dw_host_register(void* p, uint64_t bytes) {
  return (int)hipHostRegister(p, bytes, hipHostRegisterPortable);
}
extern "C" int dw_host_unregister(void* p) { return (int)hipHostUnregister(p); }

extern "C" int dw_host_registered(void* p) {
  hipPointerAttribute_t attr;
  hipError_t e = hipPointerGetAttributes(&attr, p);
  if (e != hipSuccess) { (void)hipGetLastError(); return 0; }
  return attr.type == hipMemoryTypeHost ? 1 : 0;
}

// kind: 0 H2D, 1 D2H, 2 D2D, 3 default (runtime infers)
extern "C" int dw_memcpy_async(void* dst, const void* src, uint64_t bytes, int kind, void* stream) {
  hipMemcpyKind k = kind == 0 ? hipMemcpyHostToDevice
                    : kind == 1 ? hipMemcpyDeviceToHost
                    : kind == 2 ? hipMemcpyDeviceToDevice
                                : hipMemcpyDefault;
  return (int)hipMemcpyAsync(dst, src, bytes, k, (hipStream_t)stream);
}

extern "C" int dw_stream_sync(void* stream) { return (int)hipStreamSynchronize((hipStream_t)stream); }
extern "C" int dw_event_sync(void* event) { return (int)hipEventSynchronize((hipEvent_t)event); }

// A stream whose kernels (including the runtime's blit kernels that
// implement hipMemcpyAsync to/from host memory) may only run on a subset of
// the CUs: every `stride`-th CU.  The checkpoint flush runs on such a stream
// so a multi-hundred-millisecond PCIe copy cannot occupy all 256 CUs and
// stall the training kernels on the compute stream.
extern "C" void* dw_stream_create_cumask(int stride, int* ncu_out) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return nullptr;
  const int ncu = prop.multiProcessorCount;
  const int words = (ncu + 31) / 32;
  uint32_t mask[64] = {0};
  int n = 0;
  for (int cu = 0; cu < ncu && cu < 64 * 32; ++cu) {
    if (stride <= 1 || cu % stride == 0) {
      mask[cu / 32] |= 1u << (cu % 32);
      ++n;
    }
  }
  hipStream_t s = nullptr;
  if (hipExtStreamCreateWithCUMask(&s, words, mask) != hipSuccess) return nullptr;
  if (ncu_out) *ncu_out = n;
  return (void*)s;
}

extern "C" int dw_stream_destroy(void* s) { return (int)hipStreamDestroy((hipStream_t)s); }

// Non-blocking stream (no implicit sync with the legacy null stream) with a
// priority: which = 0 lowest, 1 default, 2 highest of the device range.
extern "C" void* dw_stream_create_prio(int which, int* prio_out) {
  int lo = 0, hi = 0;
  (void)hipDeviceGetStreamPriorityRange(&lo, &hi);  // lo = least, hi = greatest priority
  const int p = which == 0 ? lo : which == 2 ? hi : (lo + hi) / 2;
  hipStream_t s = nullptr;
  if (hipStreamCreateWithPriority(&s, hipStreamNonBlocking, p) != hipSuccess) return nullptr;
  if (prio_out) *prio_out = p;
  return (void*)s;
}

// Device-side pointer for registered host memory (zero-copy stores over PCIe).
extern "C" void* dw_host_device_ptr(void* host) {
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, host, 0) != hipSuccess) { (void)hipGetLastError(); return nullptr; }
  return d;
}

// Bounded-footprint copy kernel: `blocks` workgroups stream 16-byte vectors
// (used for device->host-mapped copies where a full-chip blit would stall
// training).
__global__ void __launch_bounds__(256) stream_copy_kernel(const u32x4* __restrict__ s, u32x4* __restrict__ d,
                                                          int64_t nv) {
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < nv; i += (int64_t)gridDim.x * 256) {
    d[i] = __builtin_nontemporal_load(s + i);
  }
}
extern "C" int dw_stream_copy(void* dst, const void* src, uint64_t bytes, int blocks, void* stream) {
  if (((uintptr_t)dst | (uintptr_t)src | bytes) & 15) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(stream_copy_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const u32x4*)src,
                     (u32x4*)dst, (int64_t)(bytes >> 4));
  DW_LAUNCH_RET;
}

// ------------------------- cross-process HBM buffers ------------------------
// The checkpoint staging buffers of a local rank are allocated by its warm
// standby process and imported by the live worker (dmabuf IPC), so a snapshot
// survives the worker's death in HBM and the replacement restores with a
// device-to-device copy instead of a PCIe H2D.  Plain hipMalloc (not the
// torch caching allocator): an IPC handle names a whole allocation.
extern "C" int dw_device_malloc(uint64_t bytes, void** out) { return (int)hipMalloc(out, bytes); }
extern "C" int dw_device_free(void* p) { return (int)hipFree(p); }
extern "C" int dw_ipc_handle_size() { return (int)sizeof(hipIpcMemHandle_t); }
extern "C" int dw_ipc_get_handle(void* p, void* handle_out) {
  return (int)hipIpcGetMemHandle((hipIpcMemHandle_t*)handle_out, p);
}
extern "C" int dw_ipc_open_handle(const void* handle, void** out) {
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle, sizeof(h));
  return (int)hipIpcOpenMemHandle(out, h, hipIpcMemLazyEnablePeerAccess);
}
extern "C" int dw_ipc_close_handle(void* p) { return (int)hipIpcCloseMemHandle(p); }
extern "C" int dw_mem_get_info(uint64_t* free_b, uint64_t* total_b) {
  size_t f = 0, t = 0;
  hipError_t e = hipMemGetInfo(&f, &t);
  *free_b = f;
  *total_b = t;
  return (int)e;
}

extern "C" const char* dw_hip_error_string(int e) { return hipGetErrorString((hipError_t)e); }

extern "C" int dw_kernels_abi_version() { return 1; }

DW_PRELOAD((multi_copy_kernel<8, true>));
