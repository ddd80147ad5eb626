// Internal interface between the C ABI (icrc_capi.cpp) and the kernels
// (icrc_kernels.hip).  Not installed; the public ABI is include/roce_icrc.h.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>

namespace ricrc {

// Device table image: 7 main sets (lanes-per-packet G = 1..64, log2 index) of
// Mul(128 G), then the combine sets: [0] = Mul(-32), [1 + l] = Mul(-128 * 2^l),
// then Mul(64) (the small-frame kernel's two-chain fold), then Mul(64) once
// more as the small-frame kernel's LDS rows (Keys8, icrc_device.hpp: row e =
// 8 copies of entry e of each of the 4 tables, 128 B; the kernel copies the
// rows into the low halves of its 256-B LDS rows by LDS-DMA).
constexpr int kMaxLog2G = 6;
constexpr int kNumMainSets = kMaxLog2G + 1;
constexpr int kNumCombSets = kMaxLog2G + 1;
constexpr int kMul64Set = kNumMainSets + kNumCombSets;
constexpr int kSmallImageOff = (kMul64Set + 1) * 1024;  // words
constexpr int kSmallImageWords = 256 * 32;
constexpr int kTableWords = kSmallImageOff + kSmallImageWords;

struct IcrcArgs {
  const uint8_t* frames;
  const uint64_t* offsets;  // ragged mode
  const uint32_t* lens;     // ragged mode
  uint64_t stride;          // strided mode
  uint32_t len;             // strided mode
  uint32_t n;
  uint32_t* icrc_out;   // nullable
  uint8_t* status_out;  // nullable
  uint8_t* ok_out;      // verify mode
  const uint32_t* tables;
  // strided lane-group kernel: per-workgroup claim counters for the tail of
  // its range (epoch << 32 | next), nullable = static ranges only
  unsigned long long* claims;
  uint32_t epoch;
  // the device's service busy word (host-mapped; nullable): see announce_batch
  uint64_t* busy;
  // (uintptr_t)frames & 15, set by the launcher: the ragged kernel's compact
  // test works on offsets from the 16-byte line below `frames` (an integer
  // made from the pointer inside the kernel turned every frame load of the
  // kernel into a flat load)
  uint32_t frames_lo4;
  // ragged kernels: host-mapped word the first workgroup sets when the batch's
  // first 64-packet groups are mostly frames of at most 128 bytes (nullable);
  // the launcher picks the compact kernel for the context's next AUTO ragged
  // launch from it (icrc_kernels.hip store_tiny_hint)
  uint32_t* tiny_hint;
};

// Claim counters: per stream (up to kClaimStreams streams per context; later
// streams run without tail claims), kClaimSlots launches may be in flight at
// once (slot = epoch % kClaimSlots), each with one counter per workgroup.
constexpr int kClaimStreams = 16;
constexpr int kClaimSlots = 64;
constexpr int kMaxClaimBlocks = 1024;

// Builds the table image on the host (kTableWords words).
void build_table_image(uint32_t* out);

// Ragged launches at 8 lanes per packet run the sorted mixed-width kernel;
// `compact` (below) runs the compact kernel instead, at any lanes choice
// (include/roce_icrc.h RICRC_RAGGED_*).
constexpr bool ragged_has_compact(int log2g) { return log2g == 3; }

// Enqueues the ICRC kernel; returns a hipError_t.
hipError_t launch_icrc(const IcrcArgs& a, int log2g, bool ragged, bool verify, int num_cus,
                       hipStream_t stream, bool compact = false);

// Strided frames of at most kSmallMaxStride bytes (stride a multiple of 4):
// the lane-per-packet kernel with LDS-staged, coalesced loads.
constexpr uint32_t kSmallMaxStride = 128;
// Shortest stride it takes: a frame under 44 B (IPv4 + UDP + BTH + ICRC) is
// unusable in every kernel, and strides below hold nothing else.  The kernel
// is instantiated per chunk count ceil(stride / 16) (16-byte loads per lane
// per 64-frame batch).
constexpr uint32_t kSmallMinStride = 44;
constexpr int kSmallMinChunks = (int)((kSmallMinStride + 15u) / 16u), kSmallMaxChunks = (int)(kSmallMaxStride / 16u);
hipError_t launch_icrc_small(const IcrcArgs& a, bool verify, int num_cus, hipStream_t stream);

// Enqueues the STREAM-style read kernel (roofline denominator).
hipError_t launch_stream_read(const uint8_t* buf, uint64_t bytes, uint32_t* sink, int num_cus,
                              hipStream_t stream);

// Raises the dynamic-LDS limit of every kernel instantiation (ICRC, small
// frames, segmentation) on the current device; the C ABI calls it once per
// device (icrc_capi.cpp, prepare_device).
hipError_t prepare_kernels();
hipError_t prepare_segment_kernels();
// Raises a kernel's dynamic LDS limit and checks that it has no static LDS:
// the kernels address LDS absolutely from 0 (tables, windows, slots), so a
// static variable -- e.g. one a device-library reduction such as
// __syncthreads_or brings in -- would sit under the tables.
hipError_t set_dynamic_lds(const void* fn, int bytes);

}  // namespace ricrc

struct ricrc_seg_wr;  // include/roce_icrc.h

namespace ricrc {

struct SegArgs {
  const uint8_t* mr;
  uint64_t mr_bytes;
  const ::ricrc_seg_wr* wrs;
  uint32_t nwr;
  uint32_t pmtu;
  uint32_t npkts;
  uint8_t* frames;
  uint32_t slot;
  uint32_t* lens;  // packet -> WR map on entry (seg map kernel), frame lengths on exit
  uint32_t* icrc_out;   // nullable
  uint8_t* status_out;  // nullable
  const uint32_t* tables;
  unsigned long long* claims;  // tail-claim counters (nullable: static ranges only)
  uint32_t epoch;
  uint64_t* busy;  // the device's service busy word (nullable): see announce_batch
};

// Enqueues the packet -> WR map kernel and the segmentation kernel.
hipError_t launch_segment(const SegArgs& a, int log2g, int num_cus, hipStream_t stream);

// Enqueues the STREAM-style copy kernel (segmentation roofline denominator).
hipError_t launch_stream_copy(const uint8_t* src, uint8_t* dst, uint64_t bytes, int num_cus,
                              hipStream_t stream);

}  // namespace ricrc

namespace ricrc {

// Per-packet service (icrc_kernels.hip, icrc_service_kernel): the request /
// response slot in pinned fine-grained host memory.  Host-written words and
// GPU-written words sit on separate 128-byte lines; the frame at kSvcFrame.
struct ServiceRing {
  // host: sequence number (low 32 bits) and frame length incl. the ICRC slot
  // (high 32), published with ONE 8-byte release store after the frame, so
  // the wave learns both with one PCIe read and issues the frame's loads at
  // once (a separate length word cost a second round trip, ~1.5 us)
  uint64_t req;
  uint32_t stop;  // host: 1 = leave now
  // host: an inline request (kSvcInline, round 4) carries its frame (<= 48 B)
  // in the rest of the slot's first 64 bytes, which the wave's poll reads
  // anyway (one 64-byte load: the request needs no second PCIe round trip for
  // its bytes); `check` = svc_inline_check(seq, the 48 bytes), written with
  // the frame before req, so a poll that saw req but not all of the frame's
  // bytes (a torn read) is recognised and served from kSvcFrame instead
  uint32_t check;
  uint8_t inline_frame[48];
  uint32_t pad0[16];
  // GPU: the answer, ONE 8-byte store: ICRC (bits 0-31), status (32-39) and
  // the request's sequence number mod 2^24 (40-63) -- no fence between a
  // result and its sequence number
  uint64_t resp;
  uint32_t exited;  // GPU: 1 when the wave has left its loop
  uint32_t polls;   //      poll iterations before the last request was seen
  uint64_t t_seen;  //      real-time counter (100 MHz) when it was seen
  uint64_t t_done;  //      ... when its result was ready
  uint32_t pad1[24];
};
constexpr uint32_t kSvcSeqMask = 0xFFFFFFu;
constexpr uint32_t kSvcFrame = 1024;  // frame offset in the slot (aligned grid: 1 KiB at G = 64)
constexpr uint32_t kSvcMaxFrame = 65536;
// Burst requests (round 3): up to kSvcMaxBurst frames packed dword-aligned in
// the frame region, one descriptor each (offset from kSvcFrame | length << 32)
// and one 8-byte answer each (ICRC bits 0-31, status 32-39, verify verdict
// 40-47, the request's tag 48-63, never 0: the host zeroes the answers before
// it publishes, so an answer is complete when its tag matches, and no fence
// orders answers against a flag); the request's high word is kSvcBurst |
// (verify ? kSvcVerify : 0) | packed KiB << 16 | count.
constexpr uint32_t kSvcMaxBurst = 64;
__host__ __device__ inline uint32_t svc_burst_tag(uint32_t seq) { return (seq & 0x7FFFu) | 0x8000u; }
constexpr uint32_t kSvcBurst = 0x80000000u, kSvcVerify = 0x40000000u;
constexpr uint32_t kSvcInline = 0x20000000u;  // single frame, also in ServiceRing::inline_frame
constexpr uint32_t kSvcInlineMax = 48;
// Horner hash of the request's sequence number and the 12 dwords of the
// inline frame (zero-padded to 48 bytes), mod 2^32
__host__ __device__ inline uint32_t svc_inline_check(uint32_t seq, const uint32_t* d12) {
  uint32_t h = seq;
  for (int k = 0; k < 12; ++k) h = h * 0x9E3779B1u + d12[k];
  return h;
}
constexpr uint32_t kSvcDesc = kSvcFrame + kSvcMaxFrame;
constexpr uint32_t kSvcAns = kSvcDesc + 8 * kSvcMaxBurst;
constexpr size_t kSvcBytes = kSvcAns + 8 * kSvcMaxBurst;
static_assert(sizeof(ServiceRing) == 256, "two 128-byte lines");
static_assert(offsetof(ServiceRing, req) == 0 && offsetof(ServiceRing, stop) == 8 &&
                  offsetof(ServiceRing, check) == 12 && offsetof(ServiceRing, inline_frame) == 16,
              "the service polls req, stop, check and the inline frame with one 64-byte load");

struct ServiceArgs {
  ServiceRing* ring;  // device view of the host slot
  const uint32_t* tables;
  uint32_t served;      // last request sequence number already answered
  uint64_t idle_ticks;  // 100 MHz ticks without a request before the wave leaves
  // the device's busy word (host-mapped, 16 bytes): the real-time stamp of the
  // latest batch workgroup start on this device; the wave leaves (when no
  // request is pending) while the stamp is younger than busy_ticks
  const uint64_t* busy;
  uint64_t busy_ticks;
};

// Every service on a device shares one busy word; every batch kernel launched
// on that device stamps it (announce_batch, icrc_device.hpp), so a batch
// launched by ANY context gets the CUs that resident service waves hold
// within one poll of theirs.  20 us of the 100 MHz counter: a batch's
// workgroups start within a few microseconds of each other, and a wave
// relaunched while a batch runs only finds a CU once one of the batch's
// workgroups has finished, long after its stamp.
constexpr uint64_t kSvcBusyTicks = 2000;
constexpr size_t kBusyBytes = 128;  // one line per device

// Enqueues the service kernel (one workgroup) on `stream`.
hipError_t launch_service(const ServiceArgs& a, hipStream_t stream);

struct FaultArgs {
  uint8_t* frames;
  const uint64_t* offsets;
  const uint32_t* lens;
  uint32_t n;
  uint64_t seed;
  uint32_t rate_ppm;
  uint32_t kinds;
  uint8_t* fault_out;  // nullable
};

// Enqueues the fault-injection kernel.
hipError_t launch_faults(const FaultArgs& a, int num_cus, hipStream_t stream);

}  // namespace ricrc
