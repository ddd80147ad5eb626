// Per-packet service latency probe (round 4): where should the request slot
// live?  One resident wave polls a request word and answers into pinned host
// memory (as icrc_service_kernel does); the host publishes a request, spins on
// the answer, and times the round trip.  Variants:
//   host   : request slot in pinned coherent host memory, the wave polls it
//            over PCIe (today's service)
//   vram   : request slot in fine-grained DEVICE memory written by the host
//            through the BAR (posted PCIe writes), the wave polls local memory
// Every poll loop ends by itself after ~2 s (100 MHz real-time counter), so the
// grid always drains.  Prints one JSON line per variant (median / p99 us over
// 2000 round trips) or the reason a variant could not run.
// build: hipcc --offload-arch=gfx950 -O3 -o scratch/pingpong scratch/pingpong.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      printf("{\"error\": \"%s\", \"line\": %d}\n", hipGetErrorString(e_), __LINE__); \
      return 1;                                                                \
    }                                                                          \
  } while (0)

// req[0] = sequence number the host published; ans[0] = sequence answered
__global__ void pong(const uint32_t* req, uint32_t* ans, uint32_t n) {
  if (threadIdx.x != 0) return;
  uint32_t served = 0;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (served < n) {
    const uint32_t s = __hip_atomic_load(req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (s != served) {
      served = s;
      __hip_atomic_store(ans, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    } else if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {  // 2 s: leave
      break;
    }
  }
}

static int run(const char* name, uint32_t* req_host_view, const uint32_t* req_dev_view,
               uint32_t* ans) {
  const uint32_t n = 2000;
  __atomic_store_n(req_host_view, 0u, __ATOMIC_SEQ_CST);
  __atomic_store_n(ans, 0u, __ATOMIC_SEQ_CST);
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipLaunchKernelGGL(pong, dim3(1), dim3(64), 0, s, req_dev_view, ans, n);
  CK(hipGetLastError());
  std::vector<double> us;
  bool timed_out = false;
  for (uint32_t i = 1; i <= n; ++i) {
    const auto t0 = std::chrono::steady_clock::now();
    __atomic_store_n(req_host_view, i, __ATOMIC_RELEASE);
    __builtin_ia32_sfence();  // (device memory through the BAR is write-combined: flush)
    while (__atomic_load_n(ans, __ATOMIC_ACQUIRE) != i) {
      if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(500)) {
        timed_out = true;
        break;
      }
      __builtin_ia32_pause();
    }
    if (timed_out) break;
    us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
  }
  CK(hipStreamSynchronize(s));
  CK(hipStreamDestroy(s));
  if (timed_out || us.empty()) {
    printf("{\"variant\": \"%s\", \"error\": \"no answer within 500 ms after %zu round trips\"}\n", name,
           us.size());
    return 0;
  }
  std::sort(us.begin() + us.size() / 10, us.end());  // (the first tenth: warm-up, dropped)
  const size_t k = us.size() / 10, m = us.size() - k;
  printf("{\"variant\": \"%s\", \"round_trips\": %zu, \"median_us\": %.3f, \"p99_us\": %.3f, \"min_us\": %.3f}\n",
         name, m, us[k + m / 2], us[k + (size_t)(m * 0.99)], us[k]);
  fflush(stdout);
  return 0;
}

int main() {
  uint32_t* ans = nullptr;
  CK(hipHostMalloc((void**)&ans, 4096, hipHostMallocMapped | hipHostMallocCoherent));
  // host-memory request slot (today's service)
  uint32_t* hreq = nullptr;
  CK(hipHostMalloc((void**)&hreq, 4096, hipHostMallocMapped | hipHostMallocCoherent));
  for (int r = 0; r < 2; ++r) run("host", hreq, hreq, ans);
  // device fine-grained memory, written by the host through the BAR
  uint32_t* dreq = nullptr;
  hipError_t e = hipExtMallocWithFlags((void**)&dreq, 4096, hipDeviceMallocFinegrained);
  if (e != hipSuccess) {
    printf("{\"variant\": \"vram\", \"error\": \"hipExtMallocWithFlags: %s\"}\n", hipGetErrorString(e));
    return 0;
  }
  hipPointerAttribute_t attr;
  e = hipPointerGetAttributes(&attr, dreq);
  printf("{\"vram_ptr_attr\": \"%s\", \"type\": %d, \"host_ptr\": \"%p\", \"dev_ptr\": \"%p\"}\n",
         hipGetErrorString(e), (int)attr.type, attr.hostPointer, attr.devicePointer);
  fflush(stdout);
  // the host view: the same virtual address (large BAR) -- probe a write and a
  // read back through hipMemcpy before relying on it
  CK(hipMemset(dreq, 0, 4096));
  CK(hipDeviceSynchronize());
  volatile uint32_t* hv = dreq;
  hv[1] = 0x1234ABCDu;
  uint32_t back = 0;
  CK(hipMemcpy(&back, dreq + 1, 4, hipMemcpyDeviceToHost));
  printf("{\"vram_host_write_read_back\": \"0x%08x\"}\n", back);
  fflush(stdout);
  if (back != 0x1234ABCDu) return 0;
  for (int r = 0; r < 2; ++r) run("vram", dreq, dreq, ans);
  return 0;
}
