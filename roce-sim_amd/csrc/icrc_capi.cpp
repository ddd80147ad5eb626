// C ABI of the ICRC engine (include/roce_icrc.h): contexts, host-buffer and
// device-resident entry points, round-robin multi-GPU split.
//
// Every entry point that computes an ICRC runs the HIP kernels of
// icrc_kernels.hip on the GPU; there is no host-side CRC in this library.
#include "roce_icrc.h"

#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "gf2.hpp"
#include "icrc_internal.hpp"

struct ricrc_ctx {
  int device = -1;
  int num_cus = 0;
  int lanes = 0;  // 0 = automatic
  hipStream_t stream = nullptr;
  uint32_t* d_tables = nullptr;
  // tail-claim counters of the strided kernel: one region of kClaimSlots x
  // kMaxClaimBlocks counters per stream the context has launched on (up to
  // kClaimStreams streams).  Launches on one stream run in order, so a slot
  // is reused only after the launch 64 epochs earlier on the SAME stream has
  // finished; two streams never share a region (see claim_region).
  unsigned long long* d_claims = nullptr;
  struct ClaimRegion {
    hipStream_t stream;
    uint32_t epoch;
  };
  std::vector<ClaimRegion> claim_regions;
  // scratch for the host-buffer entry points
  uint8_t* d_frames = nullptr;
  size_t frames_cap = 0;
  uint64_t* d_offs = nullptr;
  uint32_t* d_lens = nullptr;
  uint32_t* d_icrc = nullptr;
  uint8_t* d_status = nullptr;
  uint8_t* d_ok = nullptr;
  size_t pkt_cap = 0;
  // segmentation scratch (host-buffer entry point)
  uint8_t* d_mr = nullptr;
  size_t mr_cap = 0;
  ricrc_seg_wr* d_wrs = nullptr;
  size_t wr_cap = 0;
  // small host calls (the per-packet drop-in): one pinned staging block and
  // its device twin, so a call is one H2D copy, one kernel, one D2H copy
  uint8_t* h_stage = nullptr;
  uint8_t* d_stage = nullptr;
  // per-packet service (ricrc_compute_one): request slot in pinned
  // fine-grained host memory, the stream its resident wave runs on
  ricrc::ServiceRing* svc = nullptr;
  hipStream_t svc_stream = nullptr;
  bool svc_launched = false;
  uint32_t svc_seq = 0;
  uint32_t svc_served = 0;  // last request answered (or abandoned): the wave's start point
  uint64_t* busy = nullptr;  // the device's service busy word (device_busy), once any service ran
  uint32_t svc_idle_us = 1000;  // 0 = service off (staged launch per call)
  std::chrono::steady_clock::time_point svc_last{};  // last call (the wave's idle clock)
  // multi-device host entry points (ricrc_*_batch_multi): two pinned staging
  // blocks with device twins, so the gather of one chunk overlaps the
  // previous chunk's copies and kernel (see multi_shard)
  struct Stage {
    uint8_t* h = nullptr;
    uint8_t* d = nullptr;
    hipEvent_t ev = nullptr;
  };
  Stage ms[2];
  size_t ms_frames = 0;  // frame bytes each block holds
  // the context's last batch launch per stream on a device where a service
  // has run (batch_launched / service_wait_batches)
  struct BatchEv {
    hipStream_t stream;
    hipEvent_t ev;
    uint64_t seq;  // batch_seq at its last record (slot reuse: the oldest)
  };
  std::vector<BatchEv> batch_evs;
  uint64_t batch_seq = 0;
  // ragged launches: the host-mapped hint word (tiny_hint) of the context, the
  // caller's variant (RICRC_RAGGED_*) and the one the last launch ran
  uint32_t* tiny_hint = nullptr;
  int ragged_variant = RICRC_RAGGED_AUTO;
  int last_ragged = RICRC_RAGGED_AUTO;
};

namespace {

// Dynamic-LDS limits of every kernel, raised once per device (the attribute
// is set with that device current) under a lock: contexts on several devices
// may be created from several threads.
std::mutex g_prepare_mu;
std::vector<bool> g_prepared;

hipError_t prepare_device(int device) {
  std::lock_guard<std::mutex> lk(g_prepare_mu);
  if ((size_t)device < g_prepared.size() && g_prepared[device]) return hipSuccess;
  hipError_t e = ricrc::prepare_kernels();
  if (e != hipSuccess) return e;
  if ((size_t)device >= g_prepared.size()) g_prepared.resize(device + 1, false);
  g_prepared[device] = true;
  return hipSuccess;
}

int hip_fail(hipError_t e) { return e == hipErrorOutOfMemory ? RICRC_ENOMEM : RICRC_EIO; }

// Per-device service busy word (ricrc::announce_batch): one host-mapped line
// per device, allocated by the first per-packet service on that device and
// kept until process exit.  Every batch launch on the device passes it to its
// kernel, whichever context launches, so resident service waves of OTHER
// contexts (ricrc_icrc's per-thread contexts, a gRPC pool's threads) leave
// the CUs a starting batch needs.  Before any service ran on a device the
// launches pass nullptr (nothing to announce to).
constexpr int kMaxDevices = 64;
std::atomic<uint64_t*> g_busy[kMaxDevices];
std::mutex g_busy_mu;

uint64_t* device_busy(int device) {
  return (device >= 0 && device < kMaxDevices) ? g_busy[device].load(std::memory_order_acquire)
                                                : nullptr;
}

hipError_t device_busy_init(int device, uint64_t** out) {
  *out = device_busy(device);
  if (*out || device < 0 || device >= kMaxDevices) return hipSuccess;
  std::lock_guard<std::mutex> lk(g_busy_mu);
  uint64_t* b = g_busy[device].load(std::memory_order_acquire);
  if (!b) {
    void* h = nullptr;
    hipError_t e = hipHostMalloc(&h, ricrc::kBusyBytes, hipHostMallocMapped | hipHostMallocCoherent);
    if (e != hipSuccess) return e;
    std::memset(h, 0, ricrc::kBusyBytes);
    b = (uint64_t*)h;
    g_busy[device].store(b, std::memory_order_release);
  }
  *out = b;
  return hipSuccess;
}

#define HIP_TRY(expr)                          \
  do {                                         \
    hipError_t _e = (expr);                    \
    if (_e != hipSuccess) return hip_fail(_e); \
  } while (0)

int log2_lanes(int lanes) {
  int l = 0;
  while ((1 << l) < lanes) ++l;
  return l;
}

// Lanes per packet, measured on MI355X ("Lanes per packet"):
// about 100 dwords per lane keeps the group's combine cheap while the group's
// 16G-byte aligned runs stay long -> G = 8 at 4 KiB MTU, 4 at the mixed-MTU
// mean (1.6 KiB), 2 for 64-B payloads.
int auto_log2g(uint32_t len) {
  if (len < 8) return 1;
  const uint32_t per = ((len - 4) / 4) / 100;
  if (per == 0) return 1;
  int l = 0;
  while (l < 4 && (2u << l) <= per) ++l;
  return l;
}

int pick_log2g(const ricrc_ctx* c, uint32_t typical_len) {
  return c->lanes > 0 ? log2_lanes(c->lanes) : auto_log2g(typical_len);
}

// Ragged batches are counting-sorted by iteration count inside each
// workgroup's window, so their sets are size-homogeneous and longer lane runs
// pay off: one notch more lanes than a uniform batch of the same mean length
// (mixed-MTU mean 1.6 KiB -> G = 8, measured best).  Device-resident ragged
// calls do not know the lengths on the host: they use the mixed-MTU choice.
// Host batches of tiny frames (ACKs, 48 B) run best one lane per packet:
// ragged 48-B frames G = 1 1655, G = 2 1351, G = 4 875 GiB/s (MI355X,
// scripts/explore.py u4); at 300 B G = 4 / 8 lead (3130 / 3155).
constexpr uint32_t kRaggedTypicalLen = 1632;
constexpr uint32_t kRaggedTinyLen = 128;
int ragged_log2g(const ricrc_ctx* c, uint32_t mean) {
  if (c->lanes > 0) return log2_lanes(c->lanes);
  if (mean <= kRaggedTinyLen) return 0;
  const int l = auto_log2g(mean) + 1;
  return l > 4 ? 4 : l;
}

hipStream_t pick_stream(const ricrc_ctx*, void* s) { return reinterpret_cast<hipStream_t>(s); }

int ensure_frames(ricrc_ctx* c, size_t bytes) {
  if (bytes <= c->frames_cap) return RICRC_OK;
  if (c->d_frames) (void)hipFree(c->d_frames);
  c->d_frames = nullptr;
  c->frames_cap = 0;
  size_t cap = bytes < 4096 ? 4096 : bytes;
  HIP_TRY(hipMalloc(&c->d_frames, cap));
  c->frames_cap = cap;
  return RICRC_OK;
}

int ensure_pkts(ricrc_ctx* c, size_t n) {
  if (n <= c->pkt_cap) return RICRC_OK;
  (void)hipFree(c->d_offs);
  (void)hipFree(c->d_lens);
  (void)hipFree(c->d_icrc);
  (void)hipFree(c->d_status);
  (void)hipFree(c->d_ok);
  c->d_offs = nullptr;
  c->d_lens = nullptr;
  c->d_icrc = nullptr;
  c->d_status = nullptr;
  c->d_ok = nullptr;
  c->pkt_cap = 0;
  size_t cap = n < 1024 ? 1024 : n;
  HIP_TRY(hipMalloc(&c->d_offs, cap * sizeof(uint64_t)));
  HIP_TRY(hipMalloc(&c->d_lens, cap * sizeof(uint32_t)));
  HIP_TRY(hipMalloc(&c->d_icrc, cap * sizeof(uint32_t)));
  HIP_TRY(hipMalloc(&c->d_status, cap));
  HIP_TRY(hipMalloc(&c->d_ok, cap));
  c->pkt_cap = cap;
  return RICRC_OK;
}

// Strided frames this small go to the lane-per-packet kernel (automatic lanes
// only; an explicit lanes setting forces the lane-group kernels).
bool use_small(const ricrc_ctx* c, uint64_t stride, uint32_t len) {
  return c->lanes == 0 && stride <= ricrc::kSmallMaxStride && stride >= ricrc::kSmallMinStride &&
         stride % 4 == 0 && len <= stride &&
         len >= 4 && len % 4 == 0;  // (other lengths: the lane-group kernels' slow path)
}

// Claim counters for a strided launch on stream `s`: the stream's own region
// and its next epoch, or nullptr (static ranges only, still correct) once
// kClaimStreams distinct streams have a region.  A slot of a region is shared
// only by launches 64 epochs apart on that one in-order stream, so a launch
// never finds its counters overwritten by a concurrent launch on another
// stream (which would silently drop its tail sets).
unsigned long long* claim_region(ricrc_ctx* c, hipStream_t s, uint32_t* epoch) {
  size_t r = 0;
  while (r < c->claim_regions.size() && c->claim_regions[r].stream != s) ++r;
  if (r == c->claim_regions.size()) {
    if (r >= (size_t)ricrc::kClaimStreams) return nullptr;
    c->claim_regions.push_back({s, 0u});
  }
  *epoch = ++c->claim_regions[r].epoch;  // (slot = epoch % kClaimSlots)
  return c->d_claims + r * (size_t)ricrc::kClaimSlots * ricrc::kMaxClaimBlocks;
}

// Batches in flight per device.  A resident service wave leaves when a batch
// starts on its device (announce_batch), but a caller that relaunched it at
// once put it back beside the running batch: relaunches during a batch cost
// the batch far more than the CU the wave holds (round 4, svc_contention.py:
// cfg2 kernel 1.37x with 1, 4 or 10 threads calling back to back and the wave
// relaunched per call).  So every batch launch on a device where a service
// has run records an event on its stream (one per context and stream: an
// earlier batch of the same context on another caller stream stays tracked),
// and a wave is relaunched only once every such event of the device has
// completed: per-packet calls wait while a batch runs on the device, batches
// run undisturbed.
std::mutex g_batch_mu;
std::vector<ricrc_ctx*> g_batch_ctxs;  // contexts with batch events
// Streams tracked per context.  A context on more streams reuses a slot whose
// batch has completed, else the least recently recorded one (its batch is
// then no longer waited for: at worst a relaunched wave lands beside it,
// which costs that batch time, never a result).
constexpr size_t kBatchStreams = 16;

void batch_launched(ricrc_ctx* c, hipStream_t s) {
  if (!device_busy(c->device)) return;  // no service on the device (yet): nothing to hold back
  size_t i = 0;
  while (i < c->batch_evs.size() && c->batch_evs[i].stream != s) ++i;
  if (i == c->batch_evs.size()) {
    if (i >= kBatchStreams) {
      i = kBatchStreams;
      for (size_t k = 0; k < c->batch_evs.size() && i == kBatchStreams; ++k)
        if (hipEventQuery(c->batch_evs[k].ev) == hipSuccess) i = k;
      if (i == kBatchStreams) {  // every tracked batch still runs: the oldest record
        i = 0;
        for (size_t k = 1; k < c->batch_evs.size(); ++k)
          if (c->batch_evs[k].seq < c->batch_evs[i].seq) i = k;
      }
      c->batch_evs[i].stream = s;
    } else {
      hipEvent_t ev = nullptr;
      if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return;
      std::lock_guard<std::mutex> lk(g_batch_mu);
      if (c->batch_evs.empty()) g_batch_ctxs.push_back(c);
      c->batch_evs.push_back({s, ev, 0});
    }
  }
  c->batch_evs[i].seq = ++c->batch_seq;
  (void)hipEventRecord(c->batch_evs[i].ev, s);
}

void batch_forget(ricrc_ctx* c) {
  if (c->batch_evs.empty()) return;
  {
    std::lock_guard<std::mutex> lk(g_batch_mu);
    for (size_t i = 0; i < g_batch_ctxs.size(); ++i)
      if (g_batch_ctxs[i] == c) {
        g_batch_ctxs.erase(g_batch_ctxs.begin() + (long)i);
        break;
      }
  }
  for (auto& b : c->batch_evs) (void)hipEventDestroy(b.ev);
  c->batch_evs.clear();
}

// Waits (at most kBatchWaitMax) until no batch launched through this library
// is in flight on the context's device.  (The events are queried under the
// lock: a context destroyed on another thread frees its events under it.)
constexpr auto kBatchWaitMax = std::chrono::milliseconds(200);
void service_wait_batches(const ricrc_ctx* c) {
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    bool running = false;
    {
      std::lock_guard<std::mutex> lk(g_batch_mu);
      for (const ricrc_ctx* x : g_batch_ctxs) {
        if (x->device != c->device) continue;
        for (const auto& b : x->batch_evs)
          if (hipEventQuery(b.ev) == hipErrorNotReady) {
            running = true;
            break;
          }
        if (running) break;
      }
    }
    if (!running || std::chrono::steady_clock::now() - t0 > kBatchWaitMax) return;
    for (int i = 0; i < 256; ++i) __builtin_ia32_pause();
  }
}

// The per-packet service's wave holds one CU's LDS while it runs: a context
// about to launch batch work asks it to leave first (it does within a few
// microseconds; the next ricrc_compute_one relaunches it).
void service_pause(ricrc_ctx* c) {
  if (c->svc_launched) __atomic_store_n(&c->svc->stop, 1u, __ATOMIC_RELEASE);
}

// Ragged kernel variant (include/roce_icrc.h RICRC_RAGGED_*): the compact
// kernel (icrc_compact_kernel) or the sorted window kernel
// (icrc_ragged_mixed_kernel).  A variant the caller set wins.  Under AUTO,
// host-buffer calls decide from the lengths they hold (host_ragged_variant);
// device-resident calls follow the context's learned hint: each context owns
// one word of a process-wide host-mapped block, a ragged launch's first
// workgroup stores into it whether the batch's first 64-packet groups are
// mostly small frames (store_tiny_hint), and the context's later AUTO
// launches run the compact kernel while it is 1 (launches enqueued back to
// back all read what the kernels finished before them wrote; a context's
// first one runs the sorted kernel).  The words are never freed: a kernel
// launched on a caller's stream may still write one after its context is
// destroyed (a recycled word then only steers a choice, never a result).
constexpr uint32_t kHintWords = 4096;
constexpr uint32_t kTinyFrameLen = 128;  // the compact kernel's longest frame
std::mutex g_hint_mu;
uint32_t* g_hints = nullptr;
uint32_t g_hint_next = 0;
bool g_hint_failed = false;  // the block could not be allocated: no hints in this process

uint32_t* hint_word() {
  std::lock_guard<std::mutex> lk(g_hint_mu);
  if (g_hint_failed) return nullptr;
  if (!g_hints) {
    void* h = nullptr;
    if (hipHostMalloc(&h, kHintWords * 64u, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
      g_hint_failed = true;  // (no hint: AUTO device launches run the sorted kernel, still exact)
      return nullptr;
    }
    std::memset(h, 0, kHintWords * 64u);
    g_hints = (uint32_t*)h;
  }
  return g_hints + 16u * (g_hint_next++ % kHintWords);  // (one 64-byte line each)
}

// AUTO for a batch whose lengths are on the host: the compact kernel streams
// 64-frame groups of small frames and folds any other group unsorted, so it
// is chosen when at least half of the batch's 64-frame groups hold only
// frames of at most 128 bytes (the kernels' own hint uses the same rule on
// the batch's first groups, icrc_kernels.hip store_tiny_hint).
int host_ragged_variant(const uint32_t* lens, uint32_t n) {
  uint32_t groups = 0, tiny = 0;
  for (uint32_t g = 0; g < n; g += 64, ++groups) {
    const uint32_t e = n - g < 64 ? n : g + 64;
    uint32_t k = g;
    while (k < e && lens[k] <= kTinyFrameLen) ++k;
    tiny += k == e ? 1u : 0u;
  }
  return tiny && 2u * tiny >= groups ? RICRC_RAGGED_COMPACT : RICRC_RAGGED_SORTED;
}

// `host_lens`: the batch's lengths when the caller passed them on the host
// (AUTO then decides from them), else nullptr.
int launch(ricrc_ctx* c, const uint8_t* frames, const uint64_t* offs, const uint32_t* lens,
           uint64_t stride, uint32_t len, uint32_t n, uint32_t* icrc, uint8_t* status, uint8_t* ok,
           bool ragged, bool verify, int log2g, hipStream_t s, const uint32_t* host_lens = nullptr) {
  service_pause(c);
  ricrc::IcrcArgs a{};
  a.frames = frames;
  a.offsets = offs;
  a.lens = lens;
  a.stride = stride;
  a.len = len;
  a.n = n;
  a.icrc_out = icrc;
  a.status_out = status;
  a.ok_out = ok;
  a.tables = c->d_tables;
  a.busy = device_busy(c->device);
  a.frames_lo4 = (uint32_t)((uintptr_t)frames & 15u);
  HIP_TRY(hipSetDevice(c->device));
  if (!ragged && n > 0 && use_small(c, stride, len) && ((uintptr_t)frames & 3u) == 0) {
    if (c->num_cus <= ricrc::kMaxClaimBlocks) a.claims = claim_region(c, s, &a.epoch);
    HIP_TRY(ricrc::launch_icrc_small(a, verify, c->num_cus, s));
  } else {
    if (!ragged && c->num_cus <= ricrc::kMaxClaimBlocks) a.claims = claim_region(c, s, &a.epoch);
    bool compact = false;
    if (ragged && n > 0) {
      if (!c->tiny_hint) c->tiny_hint = hint_word();
      a.tiny_hint = c->tiny_hint;  // (kept current under every variant, for AUTO)
      int v = c->ragged_variant;
      if (v == RICRC_RAGGED_AUTO)
        v = host_lens ? host_ragged_variant(host_lens, n)
            : c->tiny_hint && __atomic_load_n(c->tiny_hint, __ATOMIC_ACQUIRE) != 0u ? RICRC_RAGGED_COMPACT
                                                                                    : RICRC_RAGGED_SORTED;
      // (automatic lanes, or 8: an explicit other setting keeps its lane groups)
      compact = v == RICRC_RAGGED_COMPACT && (c->lanes == 0 || ricrc::ragged_has_compact(log2g));
    }
    HIP_TRY(ricrc::launch_icrc(a, log2g, ragged, verify, c->num_cus, s, compact));
    // (only a launch that was enqueued names the variant it ran)
    if (ragged && n > 0) c->last_ragged = compact ? RICRC_RAGGED_COMPACT : RICRC_RAGGED_SORTED;
  }
  batch_launched(c, s);
  return RICRC_OK;
}

// Mean frame length of a host length array (selects lanes per packet).
uint32_t mean_len(const uint32_t* lens, uint32_t n) {
  if (n == 0) return 0;
  uint64_t s = 0;
  for (uint32_t i = 0; i < n; ++i) s += lens[i];
  return (uint32_t)(s / n);
}

// Small host calls (the per-packet drop-in) go through one pinned staging
// block and its device twin: the caller's frames, offsets and lengths are
// packed into it ([frames | offsets | lens], then [icrc | status | ok] on the
// way back), so a call is one H2D copy, one kernel and one D2H copy instead
// of three copies in and up to three out from pageable memory: 51 -> 25 us
// per ricrc_compute_one on MI355X.  (Measured and not kept: a zero-copy
// variant, the kernel reading the mapped host block over PCIe, and polling
// hipStreamQuery instead of hipStreamSynchronize -- both the same latency;
// the floor is the launch + copy + synchronise round trip.)
constexpr size_t kStageBytes = 1u << 20;
constexpr size_t kStageMaxFrames = 256u << 10;  // larger calls use the device scratch
size_t up256(size_t x) { return (x + 255) & ~size_t(255); }

int ensure_stage(ricrc_ctx* c) {
  if (c->h_stage) return RICRC_OK;
  HIP_TRY(hipHostMalloc((void**)&c->h_stage, kStageBytes, hipHostMallocDefault));
  if (hipMalloc(&c->d_stage, kStageBytes) != hipSuccess) {
    (void)hipHostFree(c->h_stage);
    c->h_stage = nullptr;
    return RICRC_ENOMEM;
  }
  return RICRC_OK;
}

int host_ragged_staged(ricrc_ctx* c, const uint8_t* frames, size_t frames_bytes,
                       const uint64_t* offsets, const uint32_t* lens, uint32_t n,
                       uint32_t* icrc_out, uint8_t* status_out, uint8_t* ok_out, bool verify) {
  int rc = ensure_stage(c);
  if (rc) return rc;
  const size_t o_offs = up256(frames_bytes), o_lens = o_offs + up256(8ull * n);
  const size_t in_bytes = o_lens + 4ull * n;
  const size_t o_icrc = up256(in_bytes), o_st = o_icrc + up256(4ull * n), o_ok = o_st + up256(n);
  uint8_t* h = c->h_stage;
  uint8_t* d = c->d_stage;
  std::memcpy(h, frames, frames_bytes);
  std::memcpy(h + o_offs, offsets, 8ull * n);
  std::memcpy(h + o_lens, lens, 4ull * n);
  HIP_TRY(hipMemcpyAsync(d, h, in_bytes, hipMemcpyHostToDevice, c->stream));
  rc = launch(c, d, (const uint64_t*)(d + o_offs), (const uint32_t*)(d + o_lens), 0, 0, n,
              (uint32_t*)(d + o_icrc), d + o_st, verify ? d + o_ok : nullptr, true, verify,
              ragged_log2g(c, mean_len(lens, n)), c->stream, lens);
  if (rc) return rc;
  const size_t out_end = verify ? o_ok + n : o_st + n;
  HIP_TRY(hipMemcpyAsync(h + o_icrc, d + o_icrc, out_end - o_icrc, hipMemcpyDeviceToHost,
                         c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (icrc_out) std::memcpy(icrc_out, h + o_icrc, 4ull * n);
  if (status_out) std::memcpy(status_out, h + o_st, n);
  if (verify) std::memcpy(ok_out, h + o_ok, n);
  return RICRC_OK;
}

int service_burst(ricrc_ctx* c, const uint8_t* frames, const uint64_t* offsets,
                  const uint32_t* lens, uint32_t n, uint32_t* icrc_out, uint8_t* status_out,
                  uint8_t* ok_out, bool verify);
constexpr uint32_t kSvcBurstRoute = 64;  // host batches up to this many frames

int host_ragged(ricrc_ctx* c, const uint8_t* frames, size_t frames_bytes, const uint64_t* offsets,
                const uint32_t* lens, uint32_t n, uint32_t* icrc_out, uint8_t* status_out,
                uint8_t* ok_out, bool verify) {
  if (!c || (!frames && frames_bytes) || (n && (!offsets || !lens))) return RICRC_EINVAL;
  if (verify ? !ok_out : !icrc_out) return RICRC_EINVAL;
  if (n == 0) return RICRC_OK;
  // every frame must lie inside the copied buffer
  for (uint32_t i = 0; i < n; ++i)
    if (offsets[i] > frames_bytes || lens[i] > frames_bytes - offsets[i]) return RICRC_EINVAL;
  HIP_TRY(hipSetDevice(c->device));
  // a burst of up to 64 frames (64 KiB packed) goes to the resident wave
  // (automatic lanes only: an explicit lanes setting asks for the kernels)
  if (c->svc_idle_us && c->lanes == 0 && n <= kSvcBurstRoute) {
    uint64_t packed = 0;
    for (uint32_t i = 0; i < n; ++i) packed += ((uint64_t)lens[i] + 3u) & ~(uint64_t)3u;
    if (packed <= ricrc::kSvcMaxFrame) {
      const int rc = service_burst(c, frames, offsets, lens, n, icrc_out, status_out, ok_out, verify);
      if (rc != RICRC_EIO) return rc;  // (no answer within 1 s: the launch path below)
    }
  }
  if (frames_bytes <= kStageMaxFrames && 32ull * n + 1536 <= kStageBytes - up256(frames_bytes))
    return host_ragged_staged(c, frames, frames_bytes, offsets, lens, n, icrc_out, status_out,
                              ok_out, verify);
  int rc = ensure_frames(c, frames_bytes);
  if (rc) return rc;
  rc = ensure_pkts(c, n);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(c->d_frames, frames, frames_bytes, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(c->d_offs, offsets, n * sizeof(uint64_t), hipMemcpyHostToDevice,
                         c->stream));
  HIP_TRY(
      hipMemcpyAsync(c->d_lens, lens, n * sizeof(uint32_t), hipMemcpyHostToDevice, c->stream));
  rc = launch(c, c->d_frames, c->d_offs, c->d_lens, 0, 0, n, c->d_icrc, c->d_status,
              verify ? c->d_ok : nullptr, true, verify, ragged_log2g(c, mean_len(lens, n)),
              c->stream, lens);
  if (rc) return rc;
  if (icrc_out)
    HIP_TRY(hipMemcpyAsync(icrc_out, c->d_icrc, n * sizeof(uint32_t), hipMemcpyDeviceToHost,
                           c->stream));
  if (status_out)
    HIP_TRY(hipMemcpyAsync(status_out, c->d_status, n, hipMemcpyDeviceToHost, c->stream));
  if (verify) HIP_TRY(hipMemcpyAsync(ok_out, c->d_ok, n, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return RICRC_OK;
}

// Segmentation: the largest frame of a PMTU (IPv4 20 + UDP 8 + BTH 12 +
// RETHImmDt 20 + payload + ICRC 4), rounded up to whole 128-byte lines, so
// every slot starts on a line and a frame's lines are written whole.  (Round
// 3: 256-byte rounding, 4352 B at 4 KiB PMTU, left 212 B of every slot
// unwritten; the write stream over 4224-byte slots runs 6 % faster,
// scratch/seg_copy.hip: 4954 -> 5258 GB/s for the copy pattern alone.)
uint32_t seg_slot_bytes(uint32_t pmtu) { return (60u + pmtu + 4u + 127u) & ~127u; }

// Ops whose packets carry MR bytes (the rest are header-only, one packet).
bool seg_has_payload(uint32_t op) { return op <= RICRC_SEG_READ_RESPONSE; }

bool valid_pmtu(uint32_t pmtu) {
  return pmtu == 256 || pmtu == 512 || pmtu == 1024 || pmtu == 2048 || pmtu == 4096;
}

// Lanes per packet for segmentation (1 lane is not instantiated: the UDP
// checksum chunk and the header need G >= 2; G <= 16 keeps the slot grid).
int seg_log2g(const ricrc_ctx* c, uint32_t pmtu) {
  int l = c->lanes > 0 ? log2_lanes(c->lanes) : auto_log2g(((64u + pmtu + 255u) & ~255u) - 192u);
  return l < 1 ? 1 : l > 4 ? 4 : l;
}

int seg_ensure(ricrc_ctx* c, size_t mr_bytes, uint32_t nwr) {
  if (mr_bytes > c->mr_cap) {
    (void)hipFree(c->d_mr);
    c->d_mr = nullptr;
    c->mr_cap = 0;
    const size_t cap = mr_bytes < 4096 ? 4096 : mr_bytes;
    HIP_TRY(hipMalloc(&c->d_mr, cap));
    c->mr_cap = cap;
  }
  if (nwr > c->wr_cap) {
    (void)hipFree(c->d_wrs);
    c->d_wrs = nullptr;
    c->wr_cap = 0;
    const size_t cap = nwr < 256 ? 256 : nwr;
    HIP_TRY(hipMalloc(&c->d_wrs, cap * sizeof(ricrc_seg_wr)));
    c->wr_cap = cap;
  }
  return RICRC_OK;
}

int seg_launch(ricrc_ctx* c, const uint8_t* d_mr, uint64_t mr_bytes, const ricrc_seg_wr* d_wrs,
               uint32_t nwr, uint32_t pmtu, uint32_t npkts, uint8_t* d_frames, uint32_t slot,
               uint32_t* d_lens, uint32_t* d_icrc, uint8_t* d_status, hipStream_t s) {
  ricrc::SegArgs a{};
  a.mr = d_mr;
  a.mr_bytes = mr_bytes;
  a.wrs = d_wrs;
  a.nwr = nwr;
  a.pmtu = pmtu;
  a.npkts = npkts;
  a.frames = d_frames;
  a.slot = slot;
  a.lens = d_lens;
  a.icrc_out = d_icrc;
  a.status_out = d_status;
  a.tables = c->d_tables;
  a.busy = device_busy(c->device);
  if (c->num_cus <= ricrc::kMaxClaimBlocks) a.claims = claim_region(c, s, &a.epoch);
  service_pause(c);
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(ricrc::launch_segment(a, seg_log2g(c, pmtu), c->num_cus, s));
  batch_launched(c, s);
  return RICRC_OK;
}

// ---- per-packet service (see icrc_service_kernel) --------------------------

// Every context whose service may be running, so that process exit stops
// them before the HIP runtime tears down (a resident wave must not outlive
// the host memory it polls).
std::mutex g_svc_mu;
std::vector<ricrc_ctx*> g_svc_ctxs;
bool g_svc_atexit = false;

void service_stop_wait(ricrc_ctx* c) {
  if (!c->svc_launched) return;
  __atomic_store_n(&c->svc->stop, 1u, __ATOMIC_RELEASE);
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->svc_stream);
  c->svc_launched = false;
  // whatever request is still unanswered is abandoned: a later wave starts
  // after it (never answers it into a slot the host is refilling)
  c->svc_served = (uint32_t)__atomic_load_n(&c->svc->req, __ATOMIC_ACQUIRE);
}

void service_atexit() {
  std::lock_guard<std::mutex> lk(g_svc_mu);
  for (ricrc_ctx* c : g_svc_ctxs) service_stop_wait(c);
  g_svc_ctxs.clear();
}

int service_init(ricrc_ctx* c) {
  if (c->svc) return RICRC_OK;
  HIP_TRY(device_busy_init(c->device, &c->busy));
  void* h = nullptr;
  HIP_TRY(hipHostMalloc(&h, ricrc::kSvcBytes, hipHostMallocMapped | hipHostMallocCoherent));
  std::memset(h, 0, sizeof(ricrc::ServiceRing));
  hipError_t e = hipStreamCreateWithFlags(&c->svc_stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    (void)hipHostFree(h);
    return hip_fail(e);
  }
  c->svc = (ricrc::ServiceRing*)h;
  std::lock_guard<std::mutex> lk(g_svc_mu);
  g_svc_ctxs.push_back(c);
  if (!g_svc_atexit) {
    std::atexit(service_atexit);
    g_svc_atexit = true;
  }
  return RICRC_OK;
}

void service_forget(ricrc_ctx* c) {
  std::lock_guard<std::mutex> lk(g_svc_mu);
  for (size_t i = 0; i < g_svc_ctxs.size(); ++i)
    if (g_svc_ctxs[i] == c) {
      g_svc_ctxs.erase(g_svc_ctxs.begin() + (long)i);
      break;
    }
}

// (Re)launch the wave if it is not running: it left after a stop request or
// its idle timeout, or never ran.
int service_ensure(ricrc_ctx* c) {
  const auto now = std::chrono::steady_clock::now();
  if (c->svc_launched && __atomic_load_n(&c->svc->stop, __ATOMIC_ACQUIRE) == 0u &&
      __atomic_load_n(&c->svc->exited, __ATOMIC_ACQUIRE) == 0u) {
    // called again well within the idle timeout: the wave is still there
    // (no runtime query on the fast path); later, ask the stream
    if (now - c->svc_last < std::chrono::microseconds(c->svc_idle_us / 2) ||
        hipStreamQuery(c->svc_stream) == hipErrorNotReady) {
      c->svc_last = now;
      return RICRC_OK;
    }
  }
  c->svc_last = now;
  service_wait_batches(c);  // (see batch_launched)
  HIP_TRY(hipStreamSynchronize(c->svc_stream));  // a leaving wave has left
  ricrc::ServiceRing* r = c->svc;
  __atomic_store_n(&r->stop, 0u, __ATOMIC_RELAXED);
  __atomic_store_n(&r->exited, 0u, __ATOMIC_RELAXED);
  ricrc::ServiceArgs a{};
  a.ring = r;  // (unified addressing: the mapped host pointer is the device pointer)
  a.tables = c->d_tables;
  // the last request ANSWERED, not the last published: a wave relaunched
  // for a pending request (service_request) serves it first
  a.served = c->svc_served;
  a.idle_ticks = (uint64_t)c->svc_idle_us * 100u;  // 100 MHz real-time counter
  a.busy = c->busy;
  a.busy_ticks = ricrc::kSvcBusyTicks;
  std::atomic_thread_fence(std::memory_order_seq_cst);
  HIP_TRY(ricrc::launch_service(a, c->svc_stream));
  c->svc_launched = true;
  return RICRC_OK;
}

// Publishes a request whose frame bytes (and descriptors) are in the slot and
// waits for its answer word.  Returns RICRC_EIO (with the service stopped) if
// no answer came within a second -- the caller then takes the launch path.
// `answer`: the single-frame answer word (resp); a burst instead waits for
// `burst_last` (its last answer) to carry the request's tag.
int service_request(ricrc_ctx* c, uint32_t hi, uint64_t* answer, const uint64_t* burst_last = nullptr) {
  ricrc::ServiceRing* r = c->svc;
  const uint32_t seq = ++c->svc_seq == 0 ? ++c->svc_seq : c->svc_seq;  // (0 = nothing yet)
  __atomic_store_n(&r->req, ((uint64_t)hi << 32) | seq, __ATOMIC_RELEASE);
  const auto t0 = std::chrono::steady_clock::now();
  uint64_t ans = 0;
  auto answered = [&] {
    if (burst_last) {
      ans = __atomic_load_n(burst_last, __ATOMIC_ACQUIRE);
      return (uint32_t)(ans >> 48) == ricrc::svc_burst_tag(seq);
    }
    ans = __atomic_load_n(&r->resp, __ATOMIC_ACQUIRE);
    return (uint32_t)(ans >> 40) == (seq & ricrc::kSvcSeqMask);
  };
  for (uint32_t spin = 1;; ++spin) {
    if (answered()) break;
    if ((spin & 63u) == 0) {
      // the wave may have left (idle timeout, a batch starting on the device,
      // a stop) just before the request was published: once it has left and
      // the answer is still missing, launch it again -- from the last
      // ANSWERED sequence number, so it serves the pending request first
      if (__atomic_load_n(&r->exited, __ATOMIC_ACQUIRE) != 0u && !answered()) {
        c->svc_launched = false;
        const int rc = service_ensure(c);
        if (rc) {
          c->svc_served = seq;  // (abandoned)
          return rc;
        }
      }
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(1)) {
        service_stop_wait(c);  // (abandons it)
        return RICRC_EIO;
      }
    }
    __builtin_ia32_pause();
  }
  c->svc_served = seq;
  if (answer) *answer = ans;
  return RICRC_OK;
}

// One frame through the resident wave.  A frame of at most 48 bytes (ACK,
// NAK, read request, atomic ack) also rides in the slot's first 64 bytes,
// which the wave's poll reads with the request word: no second PCIe read for
// its bytes (ServiceRing::inline_frame).
int service_call(ricrc_ctx* c, const uint8_t* frame, uint32_t len, uint32_t* icrc_out,
                 uint8_t* status_out) {
  int rc = service_init(c);
  if (rc) return rc;
  rc = service_ensure(c);
  if (rc) return rc;
  std::memcpy((uint8_t*)c->svc + ricrc::kSvcFrame, frame, len);
  uint32_t hi = len;
  if (len <= ricrc::kSvcInlineMax) {
    const uint32_t next = c->svc_seq + 1 == 0 ? 1u : c->svc_seq + 1;  // (service_request's seq)
    uint32_t d12[12] = {0};
    std::memcpy(d12, frame, len);
    std::memcpy(c->svc->inline_frame, d12, sizeof d12);
    // (ordered before the request word by service_request's release store)
    __atomic_store_n(&c->svc->check, ricrc::svc_inline_check(next, d12), __ATOMIC_RELAXED);
    hi |= ricrc::kSvcInline;
  }
  uint64_t ans = 0;
  rc = service_request(c, hi, &ans);
  if (rc) return rc;
  *icrc_out = (uint32_t)ans;
  if (status_out) *status_out = (uint8_t)(ans >> 32);
  return RICRC_OK;
}

// A burst of up to kSvcMaxBurst frames (packed dword-aligned, at most
// kSvcMaxFrame bytes) through the resident wave: one request, one answer
// word per frame (icrc_internal.hpp, ServiceRing).
int service_burst(ricrc_ctx* c, const uint8_t* frames, const uint64_t* offsets,
                  const uint32_t* lens, uint32_t n, uint32_t* icrc_out, uint8_t* status_out,
                  uint8_t* ok_out, bool verify) {
  int rc = service_init(c);
  if (rc) return rc;
  rc = service_ensure(c);
  if (rc) return rc;
  if (n == 1) {  // one frame: the single-frame request (G = 64, no descriptor read)
    const uint32_t L = lens[0];
    uint32_t icrc = 0;
    uint8_t st = 0;
    rc = service_call(c, frames + offsets[0], L, &icrc, &st);
    if (rc) return rc;
    if (verify) {  // the kernels' verdict: the trailer (bytes L-4 .. L-1, little-endian)
      uint32_t t = 0;
      if (L >= 4) std::memcpy(&t, frames + offsets[0] + L - 4, 4);
      const bool good = (st & RICRC_PKT_FATAL) == 0;
      const bool ok = good && t == icrc;
      if (good && !ok) st |= RICRC_PKT_ICRC_MISMATCH;
      ok_out[0] = ok ? 1 : 0;
    }
    if (icrc_out) icrc_out[0] = icrc;
    if (status_out) status_out[0] = st;
    return RICRC_OK;
  }
  uint8_t* base = (uint8_t*)c->svc;
  uint64_t* desc = (uint64_t*)(base + ricrc::kSvcDesc);
  uint32_t pos = 0;
  for (uint32_t i = 0; i < n; ++i) {
    std::memcpy(base + ricrc::kSvcFrame + pos, frames + offsets[i], lens[i]);
    desc[i] = pos | ((uint64_t)lens[i] << 32);
    pos += (lens[i] + 3u) & ~3u;
  }
  uint64_t* res = (uint64_t*)(base + ricrc::kSvcAns);
  std::memset(res, 0, 8ull * n);
  // the last answer's tag ends the wait (the wave stores all of them with one
  // instruction); every other answer is then checked for its tag as well
  const uint32_t kib = (pos + 1023u) / 1024u;  // what the wave copies into LDS
  rc = service_request(c, ricrc::kSvcBurst | (verify ? ricrc::kSvcVerify : 0u) | (kib << 16) | n,
                       nullptr, res + (n - 1));
  if (rc) return rc;
  const uint32_t tag = ricrc::svc_burst_tag(c->svc_seq);
  for (uint32_t i = 0; i < n; ++i) {
    uint64_t v;
    for (uint32_t spin = 0;; ++spin) {  // (normally at once)
      v = __atomic_load_n(res + i, __ATOMIC_ACQUIRE);
      if ((uint32_t)(v >> 48) == tag) break;
      if (spin > (1u << 26)) return RICRC_EIO;
      __builtin_ia32_pause();
    }
    if (icrc_out) icrc_out[i] = (uint32_t)v;
    if (status_out) status_out[i] = (uint8_t)(v >> 32);
    if (verify) ok_out[i] = (uint8_t)(v >> 40);
  }
  return RICRC_OK;
}

// ---- context-free per-packet call (ricrc_icrc) -----------------------------
// A context is single-threaded, so each calling thread borrows one
// library-owned context per device.  A thread that exits hands its contexts
// back to a pool for the next thread (a gRPC pool's churn creates no more
// contexts than threads ever ran at once); pooled contexts live until process
// exit, where service_atexit stops their waves -- no HIP call runs on the
// thread-exit path.
std::mutex g_pool_mu;
std::vector<ricrc_ctx*> g_pool;

struct ThreadContexts {
  std::vector<ricrc_ctx*> ctxs;
  ~ThreadContexts() {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    for (ricrc_ctx* c : ctxs) g_pool.push_back(c);
  }
};

int thread_ctx(int device, ricrc_ctx** out) {
  static thread_local ThreadContexts t;
  for (ricrc_ctx* c : t.ctxs)
    if (c->device == device) {
      *out = c;
      return RICRC_OK;
    }
  ricrc_ctx* c = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    for (size_t i = 0; i < g_pool.size(); ++i)
      if (g_pool[i]->device == device) {
        c = g_pool[i];
        g_pool.erase(g_pool.begin() + (long)i);
        break;
      }
  }
  if (!c) {
    const int rc = ricrc_ctx_create(device, &c);
    if (rc != RICRC_OK) return rc;
  }
  t.ctxs.push_back(c);
  *out = c;
  return RICRC_OK;
}

// ---- multi-device host split (ricrc_compute/verify_batch_multi) ------------
// Packet i of the caller's batch belongs to shard i mod nctx.  Each shard is
// streamed through its context in chunks: the host gathers a chunk's frames
// (dword-aligned), offsets and lengths into a pinned block, then one H2D copy
// of the frames, one of the descriptors, the ragged kernel, and one D2H copy
// of [icrc | status | ok] go onto the context's stream.  Two blocks alternate,
// so while the GPU side of chunk k runs the host gathers chunk k + 1 and
// scatters chunk k - 1.  (Round 3 gathered a whole shard into a pageable
// std::vector per call and copied from it: no overlap, and the copies ran
// through the runtime's pageable staging.)
constexpr size_t kMultiChunkFrames = 8u << 20;
constexpr uint32_t kMultiChunkPkts = 1u << 16;
size_t multi_desc_off(size_t frames) { return up256(frames); }
size_t multi_out_off(size_t frames) {
  return multi_desc_off(frames) + up256(12ull * kMultiChunkPkts);
}
size_t multi_block(size_t frames) { return multi_out_off(frames) + 6ull * kMultiChunkPkts; }

void multi_free(ricrc_ctx* c) {
  for (auto& s : c->ms) {
    if (s.ev) (void)hipEventDestroy(s.ev);
    if (s.h) (void)hipHostFree(s.h);
    (void)hipFree(s.d);
    s = ricrc_ctx::Stage{};
  }
  c->ms_frames = 0;
}

int multi_ensure(ricrc_ctx* c, size_t frames) {
  frames = frames < kMultiChunkFrames ? kMultiChunkFrames : up256(frames);
  if (frames <= c->ms_frames) return RICRC_OK;
  multi_free(c);
  for (auto& s : c->ms) {
    hipError_t e = hipHostMalloc((void**)&s.h, multi_block(frames), hipHostMallocDefault);
    if (e == hipSuccess) e = hipMalloc(&s.d, multi_block(frames));
    if (e == hipSuccess) e = hipEventCreateWithFlags(&s.ev, hipEventDisableTiming);
    if (e != hipSuccess) {
      multi_free(c);
      return hip_fail(e);
    }
  }
  c->ms_frames = frames;
  return RICRC_OK;
}

struct MultiBatch {
  const uint8_t* frames;
  const uint64_t* offsets;
  const uint32_t* lens;
  uint64_t n;
  uint32_t stride;  // nctx: shard d holds packets d, d + stride, ...
  uint32_t* icrc_out;
  uint8_t* status_out;
  uint8_t* ok_out;
  bool verify;
};

int multi_shard_run(ricrc_ctx* c, const MultiBatch& b, uint32_t d) {
  if (d >= b.n) return RICRC_OK;
  uint32_t maxlen = 0;
  for (uint64_t i = d; i < b.n; i += b.stride) maxlen = b.lens[i] > maxlen ? b.lens[i] : maxlen;
  HIP_TRY(hipSetDevice(c->device));
  int rc = multi_ensure(c, ((size_t)maxlen + 3u) & ~(size_t)3u);
  if (rc) return rc;
  const size_t cap = c->ms_frames, o_desc = multi_desc_off(cap), o_out = multi_out_off(cap);
  struct Pending {
    uint64_t first = 0;  // shard index of the chunk's first packet
    uint32_t m = 0;
  } pend[2];
  // copy a finished chunk's answers to the caller's arrays
  auto scatter = [&](int s) {
    Pending& p = pend[s];
    if (!p.m) return RICRC_OK;
    HIP_TRY(hipEventSynchronize(c->ms[s].ev));
    const uint8_t* h = c->ms[s].h + o_out;
    const uint32_t* ic = (const uint32_t*)h;
    const uint8_t* st = h + 4ull * p.m;
    const uint8_t* ok = st + p.m;
    uint64_t i = d + p.first * b.stride;
    for (uint32_t k = 0; k < p.m; ++k, i += b.stride) {
      if (b.icrc_out) b.icrc_out[i] = ic[k];
      if (b.status_out) b.status_out[i] = st[k];
      if (b.verify) b.ok_out[i] = ok[k];
    }
    p.m = 0;
    return RICRC_OK;
  };
  const uint64_t total = (b.n - d + b.stride - 1) / b.stride;  // packets in this shard
  uint64_t next = 0;
  int s = 0;
  while (next < total) {
    rc = scatter(s);  // the block's previous chunk (two chunks ago) is done
    if (rc) return rc;
    uint8_t* h = c->ms[s].h;
    uint64_t* offs = (uint64_t*)(h + o_desc);
    uint32_t m = 0;
    size_t pos = 0;
    const uint64_t first = next;
    for (uint64_t i = d + next * b.stride; next < total && m < kMultiChunkPkts; i += b.stride) {
      const uint32_t L = b.lens[i];
      const size_t slot = ((size_t)L + 3u) & ~(size_t)3u;
      if (pos + slot > cap) break;
      std::memcpy(h + pos, b.frames + b.offsets[i], L);
      offs[m++] = pos;
      pos += slot;
      ++next;
    }
    // lengths right after the chunk's m offsets: one descriptor copy
    uint32_t* ls = (uint32_t*)(offs + m);
    for (uint32_t k = 0; k < m; ++k) ls[k] = b.lens[d + (first + k) * b.stride];
    uint8_t* dv = c->ms[s].d;
    if (pos) HIP_TRY(hipMemcpyAsync(dv, h, pos, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(dv + o_desc, h + o_desc, 12ull * m, hipMemcpyHostToDevice, c->stream));
    uint32_t* d_icrc = (uint32_t*)(dv + o_out);
    uint8_t* d_st = dv + o_out + 4ull * m;
    rc = launch(c, dv, (const uint64_t*)(dv + o_desc), (const uint32_t*)(dv + o_desc + 8ull * m), 0,
                0, m, d_icrc, d_st, b.verify ? d_st + m : nullptr, true, b.verify,
                ragged_log2g(c, (uint32_t)(pos / m)), c->stream, ls);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(h + o_out, dv + o_out, (b.verify ? 6ull : 5ull) * m,
                           hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipEventRecord(c->ms[s].ev, c->stream));
    pend[s] = {first, m};
    s ^= 1;
  }
  rc = scatter(s);
  if (rc) return rc;
  return scatter(s ^ 1);
}

// A shard that fails part-way may leave copies of the staging blocks queued
// on the context's stream: drain them, so the next call (or multi_ensure
// freeing a block) never meets a block that is still being copied.
int multi_shard(ricrc_ctx* c, const MultiBatch& b, uint32_t d) {
  const int rc = multi_shard_run(c, b, d);
  if (rc != RICRC_OK) {
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
  }
  return rc;
}

int batch_multi(ricrc_ctx** ctxs, int nctx, const uint8_t* frames, size_t frames_bytes,
                const uint64_t* offsets, const uint32_t* lens, uint32_t n, uint32_t* icrc_out,
                uint8_t* status_out, uint8_t* ok_out, bool verify) {
  if (!ctxs || nctx < 1 || (verify ? !ok_out : !icrc_out) || (n && (!frames || !offsets || !lens)))
    return RICRC_EINVAL;
  for (int d = 0; d < nctx; ++d)
    if (!ctxs[d]) return RICRC_EINVAL;
  for (uint32_t i = 0; i < n; ++i)
    if (offsets[i] > frames_bytes || lens[i] > frames_bytes - offsets[i]) return RICRC_EINVAL;
  const MultiBatch b{frames, offsets, lens, n, (uint32_t)nctx, icrc_out, status_out, ok_out, verify};
  // A context is single-threaded: shards that name the same context run one
  // after another on that context's thread.
  std::vector<ricrc_ctx*> uniq;
  std::vector<std::vector<int>> shards_of;
  for (int d = 0; d < nctx; ++d) {
    size_t u = 0;
    while (u < uniq.size() && uniq[u] != ctxs[d]) ++u;
    if (u == uniq.size()) {
      uniq.push_back(ctxs[d]);
      shards_of.emplace_back();
    }
    shards_of[u].push_back(d);
  }
  if (uniq.size() == 1)  // one context: the plain batch (its copies need no gather)
    return host_ragged(uniq[0], frames, frames_bytes, offsets, lens, n, icrc_out, status_out,
                       ok_out, verify);
  std::vector<int> rcs(nctx, RICRC_OK);
  auto run = [&](size_t u) {
    for (int d : shards_of[u]) {
      rcs[d] = multi_shard(uniq[u], b, (uint32_t)d);
      if (rcs[d]) return;
    }
  };
  std::vector<std::thread> th;
  for (size_t u = 1; u < uniq.size(); ++u) th.emplace_back(run, u);
  run(0);  // (the calling thread takes the first context)
  for (auto& t : th) t.join();
  for (int d = 0; d < nctx; ++d)
    if (rcs[d]) return rcs[d];
  return RICRC_OK;
}

}  // namespace

extern "C" {

int ricrc_abi_version(void) { return RICRC_ABI_VERSION; }

const char* ricrc_strerror(int code) {
  switch (code) {
    case RICRC_OK: return "ok";
    case RICRC_EINVAL: return "invalid argument";
    case RICRC_ENOMEM: return "out of memory";
    case RICRC_ENODEV: return "no usable gfx950 device";
    case RICRC_EIO: return "HIP runtime or kernel launch failure";
    default: return "unknown error";
  }
}

int ricrc_device_count(int* count) {
  if (!count) return RICRC_EINVAL;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  *count = n;
  return RICRC_OK;
}

int ricrc_ctx_create(int device, ricrc_ctx** out) {
  if (!out) return RICRC_EINVAL;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return RICRC_ENODEV;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return RICRC_ENODEV;
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return RICRC_ENODEV;
  if (!ricrc::self_test()) return RICRC_EIO;
  HIP_TRY(hipSetDevice(device));
  HIP_TRY(prepare_device(device));

  ricrc_ctx* c = new (std::nothrow) ricrc_ctx();
  if (!c) return RICRC_ENOMEM;
  c->device = device;
  c->num_cus = prop.multiProcessorCount;
  std::vector<uint32_t> img(ricrc::kTableWords);
  ricrc::build_table_image(img.data());
  hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipMalloc(&c->d_tables, img.size() * sizeof(uint32_t));
  const size_t claim_bytes = sizeof(unsigned long long) * ricrc::kClaimStreams *
                             ricrc::kClaimSlots * ricrc::kMaxClaimBlocks;
  if (e == hipSuccess) e = hipMalloc(&c->d_claims, claim_bytes);
  if (e == hipSuccess) e = hipMemset(c->d_claims, 0, claim_bytes);
  if (e == hipSuccess)
    e = hipMemcpy(c->d_tables, img.data(), img.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    ricrc_ctx_destroy(c);
    return hip_fail(e);
  }
  *out = c;
  return RICRC_OK;
}

void ricrc_ctx_destroy(ricrc_ctx* c) {
  if (!c) return;
  if (c->svc) {
    service_forget(c);
    service_stop_wait(c);
  }
  if (c->device >= 0) (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  batch_forget(c);
  (void)hipFree(c->d_tables);
  (void)hipFree(c->d_claims);
  (void)hipFree(c->d_frames);
  (void)hipFree(c->d_offs);
  (void)hipFree(c->d_lens);
  (void)hipFree(c->d_icrc);
  (void)hipFree(c->d_status);
  (void)hipFree(c->d_ok);
  (void)hipFree(c->d_mr);
  (void)hipFree(c->d_wrs);
  (void)hipFree(c->d_stage);
  multi_free(c);
  if (c->h_stage) (void)hipHostFree(c->h_stage);
  if (c->svc) (void)hipHostFree(c->svc);
  if (c->svc_stream) (void)hipStreamDestroy(c->svc_stream);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

int ricrc_ctx_set_lanes_per_packet(ricrc_ctx* c, int lanes) {
  if (!c || lanes < 0 || lanes > 64 || (lanes & (lanes - 1))) return RICRC_EINVAL;
  c->lanes = lanes;
  return RICRC_OK;
}

void* ricrc_ctx_stream(ricrc_ctx* c) { return c ? (void*)c->stream : nullptr; }

int ricrc_ctx_set_ragged_variant(ricrc_ctx* c, int variant) {
  if (!c || variant < RICRC_RAGGED_AUTO || variant > RICRC_RAGGED_SORTED) return RICRC_EINVAL;
  c->ragged_variant = variant;
  return RICRC_OK;
}

int ricrc_ctx_last_ragged_variant(ricrc_ctx* c, int* variant_out) {
  if (!c || !variant_out) return RICRC_EINVAL;
  *variant_out = c->last_ragged;
  return RICRC_OK;
}

int ricrc_lanes_for_len(ricrc_ctx* c, uint32_t len) {
  if (!c) return RICRC_EINVAL;
  if (use_small(c, len, len)) return 1;  // lane-per-packet kernel (strided, stride = len)
  return 1 << pick_log2g(c, len);
}

int ricrc_ctx_set_service(ricrc_ctx* c, uint32_t idle_us) {
  if (!c || idle_us > 10000000u) return RICRC_EINVAL;
  if (idle_us == 0 && c->svc) service_stop_wait(c);
  c->svc_idle_us = idle_us;
  if (c->svc_launched) service_pause(c);  // the next call relaunches with the new timeout
  return RICRC_OK;
}

int ricrc_ctx_service_times(ricrc_ctx* c, uint64_t* out3) {
  if (!c || !out3) return RICRC_EINVAL;
  if (!c->svc) {
    out3[0] = out3[1] = out3[2] = 0;
    return RICRC_OK;
  }
  out3[0] = c->svc->t_seen;
  out3[1] = c->svc->t_done;
  out3[2] = c->svc->polls;
  return RICRC_OK;
}

int ricrc_compute_one(ricrc_ctx* c, const uint8_t* frame, size_t len, uint32_t* icrc_out,
                      uint8_t* status_out) {
  if (!c || !frame || !icrc_out || len > 0xFFFFFFFFull) return RICRC_EINVAL;
  if (c->svc_idle_us && len <= ricrc::kSvcMaxFrame) {
    HIP_TRY(hipSetDevice(c->device));
    const int rc = service_call(c, frame, (uint32_t)len, icrc_out, status_out);
    if (rc != RICRC_EIO) return rc;  // (no answer within 1 s: the launch path below)
  }
  const uint64_t off = 0;
  const uint32_t l = (uint32_t)len;
  return host_ragged(c, frame, len, &off, &l, 1, icrc_out, status_out, nullptr, false);
}

int ricrc_icrc(const uint8_t* frame, size_t len, uint32_t* icrc_out, uint8_t* status_out) {
  if (!frame || !icrc_out || len > 0xFFFFFFFFull) return RICRC_EINVAL;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return RICRC_ENODEV;
  ricrc_ctx* c = nullptr;
  const int rc = thread_ctx(dev, &c);
  if (rc != RICRC_OK) return rc;
  return ricrc_compute_one(c, frame, len, icrc_out, status_out);
}

int ricrc_compute_batch(ricrc_ctx* c, const uint8_t* frames, size_t frames_bytes,
                        const uint64_t* offsets, const uint32_t* lens, uint32_t n,
                        uint32_t* icrc_out, uint8_t* status_out) {
  return host_ragged(c, frames, frames_bytes, offsets, lens, n, icrc_out, status_out, nullptr,
                     false);
}

int ricrc_verify_batch(ricrc_ctx* c, const uint8_t* frames, size_t frames_bytes,
                       const uint64_t* offsets, const uint32_t* lens, uint32_t n, uint8_t* ok_out,
                       uint32_t* icrc_out, uint8_t* status_out) {
  return host_ragged(c, frames, frames_bytes, offsets, lens, n, icrc_out, status_out, ok_out,
                     true);
}

int ricrc_compute_strided(ricrc_ctx* c, const uint8_t* frames, uint64_t stride, uint32_t len,
                          uint32_t n, uint32_t* icrc_out, uint8_t* status_out) {
  if (!c || !icrc_out || (n && !frames) || (n > 1 && stride < len)) return RICRC_EINVAL;
  if (n == 0) return RICRC_OK;
  const size_t bytes = (size_t)(n - 1) * stride + len;
  HIP_TRY(hipSetDevice(c->device));
  int rc = ensure_frames(c, bytes);
  if (rc) return rc;
  rc = ensure_pkts(c, n);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(c->d_frames, frames, bytes, hipMemcpyHostToDevice, c->stream));
  rc = launch(c, c->d_frames, nullptr, nullptr, stride, len, n, c->d_icrc, c->d_status, nullptr,
              false, false, pick_log2g(c, len), c->stream);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(icrc_out, c->d_icrc, n * sizeof(uint32_t), hipMemcpyDeviceToHost,
                         c->stream));
  if (status_out)
    HIP_TRY(hipMemcpyAsync(status_out, c->d_status, n, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return RICRC_OK;
}

int ricrc_compute_batch_multi(ricrc_ctx** ctxs, int nctx, const uint8_t* frames,
                              size_t frames_bytes, const uint64_t* offsets, const uint32_t* lens,
                              uint32_t n, uint32_t* icrc_out, uint8_t* status_out) {
  return batch_multi(ctxs, nctx, frames, frames_bytes, offsets, lens, n, icrc_out, status_out,
                     nullptr, false);
}

int ricrc_verify_batch_multi(ricrc_ctx** ctxs, int nctx, const uint8_t* frames,
                             size_t frames_bytes, const uint64_t* offsets, const uint32_t* lens,
                             uint32_t n, uint8_t* ok_out, uint32_t* icrc_out,
                             uint8_t* status_out) {
  return batch_multi(ctxs, nctx, frames, frames_bytes, offsets, lens, n, icrc_out, status_out,
                     ok_out, true);
}

int ricrc_host_register(void* ptr, size_t bytes) {
  if (!ptr || !bytes) return RICRC_EINVAL;
  HIP_TRY(hipHostRegister(ptr, bytes, hipHostRegisterDefault));
  return RICRC_OK;
}

int ricrc_host_unregister(void* ptr) {
  if (!ptr) return RICRC_EINVAL;
  HIP_TRY(hipHostUnregister(ptr));
  return RICRC_OK;
}

int ricrc_compute_batch_dev(ricrc_ctx* c, const uint8_t* d_frames, const uint64_t* d_offsets,
                            const uint32_t* d_lens, uint32_t n, uint32_t* d_icrc,
                            uint8_t* d_status, void* stream) {
  if (!c || !d_icrc || (n && (!d_frames || !d_offsets || !d_lens))) return RICRC_EINVAL;
  // lanes per packet for ragged device batches: the context setting, else the
  // 1 KiB-MTU choice (lengths are on the device; no host round trip)
  return launch(c, d_frames, d_offsets, d_lens, 0, 0, n, d_icrc, d_status, nullptr, true, false,
                ragged_log2g(c, kRaggedTypicalLen), pick_stream(c, stream));
}

int ricrc_verify_batch_dev(ricrc_ctx* c, const uint8_t* d_frames, const uint64_t* d_offsets,
                           const uint32_t* d_lens, uint32_t n, uint8_t* d_ok, uint32_t* d_icrc,
                           uint8_t* d_status, void* stream) {
  if (!c || !d_ok || (n && (!d_frames || !d_offsets || !d_lens))) return RICRC_EINVAL;
  return launch(c, d_frames, d_offsets, d_lens, 0, 0, n, d_icrc, d_status, d_ok, true, true,
                ragged_log2g(c, kRaggedTypicalLen), pick_stream(c, stream));
}

int ricrc_compute_strided_dev(ricrc_ctx* c, const uint8_t* d_frames, uint64_t stride, uint32_t len,
                              uint32_t n, uint32_t* d_icrc, uint8_t* d_status, void* stream) {
  if (!c || !d_icrc || (n && !d_frames) || (n > 1 && stride < len)) return RICRC_EINVAL;
  return launch(c, d_frames, nullptr, nullptr, stride, len, n, d_icrc, d_status, nullptr, false,
                false, pick_log2g(c, len), pick_stream(c, stream));
}

int ricrc_verify_strided_dev(ricrc_ctx* c, const uint8_t* d_frames, uint64_t stride, uint32_t len,
                             uint32_t n, uint8_t* d_ok, uint32_t* d_icrc, uint8_t* d_status,
                             void* stream) {
  if (!c || !d_ok || (n && !d_frames) || (n > 1 && stride < len)) return RICRC_EINVAL;
  return launch(c, d_frames, nullptr, nullptr, stride, len, n, d_icrc, d_status, d_ok, false, true,
                pick_log2g(c, len), pick_stream(c, stream));
}

int ricrc_stream_read_dev(ricrc_ctx* c, const uint8_t* d_buf, uint64_t bytes, uint32_t* d_sink,
                          void* stream) {
  if (!c || !d_buf || !d_sink || (bytes & 15)) return RICRC_EINVAL;
  HIP_TRY(hipSetDevice(c->device));
  service_pause(c);
  HIP_TRY(ricrc::launch_stream_read(d_buf, bytes, d_sink, c->num_cus, pick_stream(c, stream)));
  return RICRC_OK;
}

int ricrc_segment_plan(ricrc_seg_wr* wrs, uint32_t nwr, uint32_t pmtu, uint32_t* npkts_out,
                       uint32_t* slot_bytes_out) {
  if ((nwr && !wrs) || !npkts_out || !valid_pmtu(pmtu)) return RICRC_EINVAL;
  uint64_t total = 0;
  for (uint32_t i = 0; i < nwr; ++i) {
    if (wrs[i].op >= RICRC_SEG_NUM_OPS) return RICRC_EINVAL;
    wrs[i].first_pkt = (uint32_t)total;
    // Util.compute_wr_pkt_num (src/roce_util.py:183-185); header-only ops
    // (read request, atomics, ACK/NAK, atomic ack) are one packet each
    total += !seg_has_payload(wrs[i].op) ? 1
             : wrs[i].length              ? ((uint64_t)wrs[i].length + pmtu - 1) / pmtu
                                          : 1;
    if (total > 0xFFFFFFFFull) return RICRC_EINVAL;
  }
  *npkts_out = (uint32_t)total;
  if (slot_bytes_out) *slot_bytes_out = seg_slot_bytes(pmtu);
  return RICRC_OK;
}

int ricrc_segment(ricrc_ctx* c, const uint8_t* mr, size_t mr_bytes, const ricrc_seg_wr* wrs,
                  uint32_t nwr, uint32_t pmtu, uint8_t* frames, size_t frames_bytes,
                  uint32_t* lens, uint32_t* icrc_out, uint8_t* status_out) {
  if (!c || (mr_bytes && !mr) || (nwr && !wrs) || !valid_pmtu(pmtu)) return RICRC_EINVAL;
  // re-plan a copy: the caller's first_pkt must match, every WR must lie in the MR
  std::vector<ricrc_seg_wr> plan(wrs, wrs + nwr);
  uint32_t npkts = 0, slot = 0;
  int rc = ricrc_segment_plan(plan.data(), nwr, pmtu, &npkts, &slot);
  if (rc) return rc;
  for (uint32_t i = 0; i < nwr; ++i)
    if (plan[i].first_pkt != wrs[i].first_pkt ||
        (seg_has_payload(wrs[i].op) &&
         (wrs[i].mr_offset > mr_bytes || wrs[i].length > mr_bytes - wrs[i].mr_offset)))
      return RICRC_EINVAL;
  if (npkts == 0) return RICRC_OK;
  if (!frames || !lens || frames_bytes < (size_t)npkts * slot) return RICRC_EINVAL;
  HIP_TRY(hipSetDevice(c->device));
  rc = seg_ensure(c, mr_bytes, nwr);
  if (rc) return rc;
  rc = ensure_frames(c, (size_t)npkts * slot);
  if (rc) return rc;
  rc = ensure_pkts(c, npkts);
  if (rc) return rc;
  if (mr_bytes) HIP_TRY(hipMemcpyAsync(c->d_mr, mr, mr_bytes, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(c->d_wrs, plan.data(), nwr * sizeof(ricrc_seg_wr), hipMemcpyHostToDevice,
                         c->stream));
  rc = seg_launch(c, c->d_mr, mr_bytes, c->d_wrs, nwr, pmtu, npkts, c->d_frames, slot, c->d_lens,
                  c->d_icrc, c->d_status, c->stream);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(frames, c->d_frames, (size_t)npkts * slot, hipMemcpyDeviceToHost,
                         c->stream));
  HIP_TRY(hipMemcpyAsync(lens, c->d_lens, npkts * sizeof(uint32_t), hipMemcpyDeviceToHost,
                         c->stream));
  if (icrc_out)
    HIP_TRY(hipMemcpyAsync(icrc_out, c->d_icrc, npkts * sizeof(uint32_t), hipMemcpyDeviceToHost,
                           c->stream));
  if (status_out)
    HIP_TRY(hipMemcpyAsync(status_out, c->d_status, npkts, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return RICRC_OK;
}

int ricrc_segment_dev(ricrc_ctx* c, const uint8_t* d_mr, uint64_t mr_bytes,
                      const ricrc_seg_wr* d_wrs, uint32_t nwr, uint32_t pmtu, uint32_t npkts,
                      uint8_t* d_frames, uint32_t slot_bytes, uint32_t* d_lens, uint32_t* d_icrc,
                      uint8_t* d_status, void* stream) {
  if (!c || !valid_pmtu(pmtu) || (nwr && !d_wrs) || (mr_bytes && !d_mr)) return RICRC_EINVAL;
  if (npkts == 0) return RICRC_OK;
  if (!d_frames || !d_lens || (slot_bytes & 127u) || slot_bytes < seg_slot_bytes(pmtu) ||
      ((uintptr_t)d_frames & 255u))
    return RICRC_EINVAL;
  return seg_launch(c, d_mr, mr_bytes, d_wrs, nwr, pmtu, npkts, d_frames, slot_bytes, d_lens,
                    d_icrc, d_status, pick_stream(c, stream));
}

int ricrc_inject_faults_dev(ricrc_ctx* c, uint8_t* d_frames, const uint64_t* d_offsets,
                            const uint32_t* d_lens, uint32_t n, uint64_t seed, uint32_t rate_ppm,
                            uint32_t kinds, uint8_t* d_fault_out, void* stream) {
  if (!c || rate_ppm > 1000000u || (n && (!d_frames || !d_offsets || !d_lens))) return RICRC_EINVAL;
  ricrc::FaultArgs a{};
  a.frames = d_frames;
  a.offsets = d_offsets;
  a.lens = d_lens;
  a.n = n;
  a.seed = seed;
  a.rate_ppm = rate_ppm;
  a.kinds = kinds;
  a.fault_out = d_fault_out;
  HIP_TRY(hipSetDevice(c->device));
  service_pause(c);
  HIP_TRY(ricrc::launch_faults(a, c->num_cus, pick_stream(c, stream)));
  return RICRC_OK;
}

int ricrc_stream_copy_dev(ricrc_ctx* c, const uint8_t* d_src, uint8_t* d_dst, uint64_t bytes,
                          void* stream) {
  if (!c || !d_src || !d_dst || (bytes & 15)) return RICRC_EINVAL;
  HIP_TRY(hipSetDevice(c->device));
  service_pause(c);
  HIP_TRY(ricrc::launch_stream_copy(d_src, d_dst, bytes, c->num_cus, pick_stream(c, stream)));
  return RICRC_OK;
}

}  // extern "C"
