// stft.hip — frame-parallel STFT -> power -> Slaney mel -> dB for every frame of
// a batch of sequences (librosa.feature.melspectrogram + power_to_db inside
// onset_strength; oracle/ncref.py mel_db).  Shared by the per-window tempo path
// (hop 512, tempo.py:44 via librosa.onset.onset_strength) and the full-signal
// IBI pass (hop 64, tempo.py:139).
//
// MI355X layout: a workgroup of SM_WAVES = 16 waves, one STFT frame per wave (the
// 2048-point real frame is a 1024-point complex wave FFT, radix 16.16.4 whose two
// exchanges each pass through a 4.2 KB LDS slot in two halves).  Workgroups are persistent and walk a CONTIGUOUS range of
// frames, so the 4x frame overlap (n_fft 2048 / hop 512) is served from the
// XCD's own L2.  Twiddles (2048 entries), the mel CSR weights and their row
// descriptors are staged once per workgroup in LDS.  Per frame the kernel writes
// the 128 dB values, the frame max (the power_to_db top_db clamp needs the
// sequence max) and, optionally, the f64 energy of the hop-length slice the
// frame is centred on (the io.slice_windows energy, io.py:38-40, fused into the
// same HBM read).
#include <algorithm>

#include "nc_block.h"
#include "nc_engine.h"
#include "nc_piptrack.h"

#include "stft_args.h"

namespace nc {

// Measured and not kept (rounds 2-3): two workgroups per CU (the same alone,
// slower in the step: the extra workgroups queue behind the chroma stream's kernels); the
// mel weights read through L1 instead of LDS (16 waves: 625 against 579 us per 560 windows);
// the Hann window through L1 (607 against 566 us).
constexpr int SM_HANN2 = 1024;  // float2 elements of the staged Hann window
// 16 waves (four per SIMD), one frame each, in half-size exchange slots (round 4; the round-3
// kernel ran 14 waves in full 8.4 KB slots)
constexpr int SM_WAVES = 16;
constexpr int SM_THREADS = SM_WAVES * 64;
constexpr int SM_HALF = 528;  // float2 per half-size slot: 512 exchange elements + pads
// LDS requested per workgroup: 150 KB, so no chroma-chain workgroup shares a CU with the STFT (the
// kernel needs 105 KB; with the rest free the decimator co-resided and its span per step went
// 1.2 -> 2.1 ms, the step no faster: tools/ab_bench.sh, profiles/r4_stft_lds_pad_ab.txt).  Round 5
// tried letting the octave 0-2 CQT (MFMA-bound, 38 KB, 219 VGPRs) share the STFT's CUs: 12 STFT
// waves at 96 VGPRs with a 120 KB reserve ran the step at 9.36-10.40 ms against 9.22-9.61 (16 waves,
// 150 KB) and 16 waves with a 120 KB reserve at 9.31-9.72 (profiles/r5_stft_coresidency_ab.txt)
constexpr size_t SM_LDS_RESERVE = 150 * 1024;
#ifndef SM_NOEN_
#define SM_NOEN_ 0  // timing probe: the frame energies left out even when asked for (outputs wrong)
#endif
// Round 6 (profiles/r6_stft_sync_*.txt): with a static interleave (wave w: frames
// 16 G + w) the free-running waves of a workgroup drift apart by tens of frame groups, so the 4x
// frame overlap is re-fetched from beyond the L2: reads 1.62x the algorithmic bytes.  Keeping them together with a bare s_barrier every 8 groups
// (SM_SYNC_=8) cuts the reads to 1.02x, but costs 3.6 % of the kernel's time (457.4 against 441.3 us
// per 560 windows; every 32 groups: 1.44x, +1.2 %; __syncthreads every 1-32 groups: +4-22 %); each
// wave walking its own contiguous run (a probe since removed) reads 1.96x and is 1-10 % slower.  The kernel is
// not bound by its HBM bytes, so the waves stay free-running.
#ifndef SM_SYNC_
#define SM_SYNC_ 0  // probe (static interleave only): a barrier every SM_SYNC_ frame groups
#endif
// The fix (round 6): the sixteen waves take the workgroup's frames one at a time from an LDS
// counter (SM_DYN_, default), so the frames in flight are always the sixteen most recently taken,
// whatever the waves' relative speeds: reads 1.62x -> 1.00x algorithmic, 443.1 -> 399.8 us per 560
// windows (-9.8 %), the wave that finishes first no longer idles at the end of the range, outputs
// bit-identical (profiles/r6_stft_dyn_var_bench.txt).  SM_DYN_=0 restores the static interleave.
#ifndef SM_DYN_
#define SM_DYN_ 1
#endif
using SmTw = StagedTw<1024>;  // per-stage twiddle table in LDS (conflict-free reads)

// Mel band loops with compile-time trip counts, unrolled in load batches: 562-576 against
// 577-596 us per 560 windows (round 3, same session), bit-identical.
// float4 steps of the short / long band of a lane (nc_tables.cpp): 3 / 14 at 22 050 Hz; the 4 / 17
// instance serves contexts built for other rates (16-48 kHz, nc_create_rate)
constexpr int kMelJ0 = 3, kMelJ1 = 14;
constexpr int kMelJ0w = 4, kMelJ1w = 17;
constexpr int kMelB = 7;                // steps per load batch

// acc = the fmaf chain of mel_loop over j < nj (< J), in the same order: batches of kMelB
// steps, loads first, then the chain.  Every lane runs all J steps: past its band the weights
// are the table's zero padding, and fmaf(0, p, acc) == acc for the finite p it then reads
// (the power, exchange data, or the slot's zeroed pads), so the sum is bit-identical to the
// per-lane trip count nj, without the 17 exec-masked branches per frame it cost (553 -> 520 us
// per 560 windows, round 3)
template <int J>
__device__ __forceinline__ void mel_unrolled(const float* pw, const float4* w4, int lo, int nj, int lane, float& acc) {
#pragma unroll
  for (int j0 = 0; j0 < J; j0 += kMelB) {
    float4 p[kMelB], w[kMelB];
#pragma unroll
    for (int j = 0; j < kMelB; ++j)
      if (j0 + j < J) {
        p[j] = *reinterpret_cast<const float4*>(pw + lo + 4 * (j0 + j));
        w[j] = w4[(j0 + j) * 64 + lane];
      }
#pragma unroll
    for (int j = 0; j < kMelB; ++j)
      if (j0 + j < J) acc = fmaf(w[j].w, p[j].w, fmaf(w[j].z, p[j].z, fmaf(w[j].y, p[j].y, fmaf(w[j].x, p[j].x, acc))));
  }
}

__device__ __forceinline__ int seq_of_frame(const int64_t* base, int n, int64_t g) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (base[mid] <= g) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

__host__ __device__ __forceinline__ int al4(int n) { return (n + 3) & ~3; }

// mel lane-slot descriptors staged in LDS (a global read at the mel step exposes its latency):
// lo4 | nj4 << 11 | band << 16 per (slot, lane)
constexpr int SM_MT = 128;
__host__ __device__ __forceinline__ int mel_pack(int lo4, int nj4, int band) { return lo4 | (nj4 << 11) | (band << 16); }

size_t stft_mel_lds_bytes(int mel_j) {
  return (size_t)al4(SmTw::size) * sizeof(float2) + (size_t)mel_j * 64 * sizeof(float4) +
         (size_t)SM_HANN2 * sizeof(float2) + (size_t)SM_MT * sizeof(int) +
         (size_t)SM_WAVES * SM_HALF * sizeof(float2);
}

// ------------------------------------------------------------------------------ half-size slots
// The exchanges of the 1024-point FFT in two halves of 512 elements each, through a slot of
// SM_HALF float2 (4.2 KB instead of 8.4), so 16 waves (four per SIMD) fit beside the tables
// where 14 full slots did (round 4; an occupancy probe with overlapping slots ran 434 against
// 477 us per 560 windows at 16 against 14 waves, 502 us at 20).  Every frame's arithmetic and
// its order are those of the full-slot kernel: results are bit-identical.
//
// Exchange 1 (stage 1 -> stage 2).  Lane l runs stage-1 butterfly j = sm_j1(l) over the samples
// x[2 (j + 64 r)], outputs r' = 0..15.  Half A holds the outputs r' < 8 of every butterfly, at
// 8 j + j / 4 + r'; half B the outputs r' >= 8 the same way.  Stage-2 butterfly j2 = sm_j2(l)
// reads elements j2 + 64 r, i.e. output r' = j2 % 16 of butterflies j2 / 16 + 4 r: lanes 0-31
// have j2 % 16 < 8 and read half A, lanes 32-63 half B, both at l % 32 + 33 r.  The 16-lane
// write groups and the 32-lane read groups are bank-conflict free by construction (the j / 4
// pad spreads a write group's rows over 16 distinct banks; a read group covers 32 consecutive
// elements).
// Exchange 2 (stage 2 -> the mirror-paired last stage).  Stage-2 butterfly j2 writes output r
// at block b = j2 / 16, in-block index J = j2 % 16 + 16 r; half A holds J < 128 at
// sm_boff(b) + J (blocks at 0, 136, 264, 400: a write group's two blocks 8 banks apart, the
// four blocks inside 528 elements), half B J >= 128 at the same place less 128.  The last stage's lane l
// reads J in its mirror set {l, 128 - l | 128 + l, 256 - l}: two of them in each half, every
// lane in both halves.
// After the split the power spectrum [0, 1025) fills the slot (1056 floats); piptrack runs after
// the mel step, its |X| stencil bins written over the power in place and its peak bins at 512.
__device__ __forceinline__ int sm_j1(int l) {  // stage-1 butterfly of lane l (write groups conflict free)
  const int G = l >> 4, i = l & 15;
  return 4 * (8 * (G >> 1) + (i >> 1)) + (i & 1) + 2 * (G & 1);
}
__device__ __forceinline__ int sm_j2(int l) {  // stage-2 butterfly of lane l (lanes 0-31: half A)
  return (l & 7) + 8 * (l >> 5) + 16 * ((l & 31) >> 3);
}
__host__ __device__ constexpr int sm_boff(int b) { return b == 0 ? 0 : b == 1 ? 136 : b == 2 ? 264 : 400; }
constexpr int kPipKpkHalf = 512;  // float offset of the compacted piptrack peak bins in a half slot
static_assert(kPipKpkHalf >= kPipHi - kPipLo + 3 && kPipKpkHalf + (kPipHi - kPipLo + 1) <= 2 * SM_HALF,
              "piptrack half-slot layout");

#define NC_W_(v, o) "ds_write_b64 %[wb], %[" #v "] offset:" #o "\n\t"
#define NC_R_(d, b, o) "ds_read_b64 %[" #d "], %[" #b "] offset:" #o "\n\t"

// Exchange 1: v[r'] (stage-1 outputs) in, u[r] = element sm_j2(l) + 64 r out.  One asm block:
// half A written, read by lanes 0-31 (EXEC upper half off), half B written over it (the LDS runs a
// wave's operations in order, so the reads have their data), read by lanes 32-63, one wait.
__device__ __forceinline__ void sm_exchange1(const float2 (&v)[16], float2 (&u)[16], uint32_t wb, uint32_t rb) {
  nc_f2v i0 = {v[0].x, v[0].y}, i1 = {v[1].x, v[1].y}, i2 = {v[2].x, v[2].y}, i3 = {v[3].x, v[3].y};
  nc_f2v i4 = {v[4].x, v[4].y}, i5 = {v[5].x, v[5].y}, i6 = {v[6].x, v[6].y}, i7 = {v[7].x, v[7].y};
  nc_f2v i8 = {v[8].x, v[8].y}, i9 = {v[9].x, v[9].y}, i10 = {v[10].x, v[10].y}, i11 = {v[11].x, v[11].y};
  nc_f2v i12 = {v[12].x, v[12].y}, i13 = {v[13].x, v[13].y}, i14 = {v[14].x, v[14].y}, i15 = {v[15].x, v[15].y};
  nc_f2v d0, d1, d2, d3, d4, d5, d6, d7, d8, d9, d10, d11, d12, d13, d14, d15;
  unsigned long long sv;
  asm volatile(
      NC_W_(i0, 0) NC_W_(i1, 8) NC_W_(i2, 16) NC_W_(i3, 24) NC_W_(i4, 32) NC_W_(i5, 40) NC_W_(i6, 48) NC_W_(i7, 56)
      "s_mov_b64 %[sv], exec\n\t"
      "s_mov_b32 exec_hi, 0\n\t"
      NC_R_(d0, rb, 0) NC_R_(d1, rb, 264) NC_R_(d2, rb, 528) NC_R_(d3, rb, 792) NC_R_(d4, rb, 1056)
      NC_R_(d5, rb, 1320) NC_R_(d6, rb, 1584) NC_R_(d7, rb, 1848) NC_R_(d8, rb, 2112) NC_R_(d9, rb, 2376)
      NC_R_(d10, rb, 2640) NC_R_(d11, rb, 2904) NC_R_(d12, rb, 3168) NC_R_(d13, rb, 3432) NC_R_(d14, rb, 3696)
      NC_R_(d15, rb, 3960)
      "s_mov_b64 exec, %[sv]\n\t"
      NC_W_(i8, 0) NC_W_(i9, 8) NC_W_(i10, 16) NC_W_(i11, 24) NC_W_(i12, 32) NC_W_(i13, 40) NC_W_(i14, 48)
      NC_W_(i15, 56)
      "s_mov_b32 exec_lo, 0\n\t"
      NC_R_(d0, rb, 0) NC_R_(d1, rb, 264) NC_R_(d2, rb, 528) NC_R_(d3, rb, 792) NC_R_(d4, rb, 1056)
      NC_R_(d5, rb, 1320) NC_R_(d6, rb, 1584) NC_R_(d7, rb, 1848) NC_R_(d8, rb, 2112) NC_R_(d9, rb, 2376)
      NC_R_(d10, rb, 2640) NC_R_(d11, rb, 2904) NC_R_(d12, rb, 3168) NC_R_(d13, rb, 3432) NC_R_(d14, rb, 3696)
      NC_R_(d15, rb, 3960)
      "s_mov_b64 exec, %[sv]\n\t"
      "s_waitcnt lgkmcnt(0)"
      : [d0] "=&v"(d0), [d1] "=&v"(d1), [d2] "=&v"(d2), [d3] "=&v"(d3), [d4] "=&v"(d4), [d5] "=&v"(d5),
        [d6] "=&v"(d6), [d7] "=&v"(d7), [d8] "=&v"(d8), [d9] "=&v"(d9), [d10] "=&v"(d10), [d11] "=&v"(d11),
        [d12] "=&v"(d12), [d13] "=&v"(d13), [d14] "=&v"(d14), [d15] "=&v"(d15), [sv] "=&s"(sv)
      : [wb] "v"(wb), [rb] "v"(rb), [i0] "v"(i0), [i1] "v"(i1), [i2] "v"(i2), [i3] "v"(i3), [i4] "v"(i4),
        [i5] "v"(i5), [i6] "v"(i6), [i7] "v"(i7), [i8] "v"(i8), [i9] "v"(i9), [i10] "v"(i10), [i11] "v"(i11),
        [i12] "v"(i12), [i13] "v"(i13), [i14] "v"(i14), [i15] "v"(i15)
      : "memory");
  const nc_f2v d[16] = {d0, d1, d2, d3, d4, d5, d6, d7, d8, d9, d10, d11, d12, d13, d14, d15};
#pragma unroll
  for (int r = 0; r < 16; ++r) u[r] = make_float2(d[r].x, d[r].y);
}

// Exchange 2: v[r] (stage-2 outputs) in, o[4 m + r3] = element mirror_J(l, m) + 256 r3 out;
// half A (J < 128: m = 0, 1) then half B (m = 2, 3), all lanes in both, one wait.  Read bases
// rb_m = the lane's in-half index of mirror_J(l, m); block r3 at sm_boff(r3).
__device__ __forceinline__ void sm_exchange2(const float2 (&v)[16], float2 (&o)[16], uint32_t wb, uint32_t r0,
                                             uint32_t r1, uint32_t r2, uint32_t r3) {
  nc_f2v i0 = {v[0].x, v[0].y}, i1 = {v[1].x, v[1].y}, i2 = {v[2].x, v[2].y}, i3 = {v[3].x, v[3].y};
  nc_f2v i4 = {v[4].x, v[4].y}, i5 = {v[5].x, v[5].y}, i6 = {v[6].x, v[6].y}, i7 = {v[7].x, v[7].y};
  nc_f2v i8 = {v[8].x, v[8].y}, i9 = {v[9].x, v[9].y}, i10 = {v[10].x, v[10].y}, i11 = {v[11].x, v[11].y};
  nc_f2v i12 = {v[12].x, v[12].y}, i13 = {v[13].x, v[13].y}, i14 = {v[14].x, v[14].y}, i15 = {v[15].x, v[15].y};
  nc_f2v d0, d1, d2, d3, d4, d5, d6, d7, d8, d9, d10, d11, d12, d13, d14, d15;
  asm volatile(
      NC_W_(i0, 0) NC_W_(i1, 128) NC_W_(i2, 256) NC_W_(i3, 384) NC_W_(i4, 512) NC_W_(i5, 640) NC_W_(i6, 768)
      NC_W_(i7, 896)
      NC_R_(d0, r0, 0) NC_R_(d1, r0, 1088) NC_R_(d2, r0, 2112) NC_R_(d3, r0, 3200)
      NC_R_(d4, r1, 0) NC_R_(d5, r1, 1088) NC_R_(d6, r1, 2112) NC_R_(d7, r1, 3200)
      NC_W_(i8, 0) NC_W_(i9, 128) NC_W_(i10, 256) NC_W_(i11, 384) NC_W_(i12, 512) NC_W_(i13, 640) NC_W_(i14, 768)
      NC_W_(i15, 896)
      NC_R_(d8, r2, 0) NC_R_(d9, r2, 1088) NC_R_(d10, r2, 2112) NC_R_(d11, r2, 3200)
      NC_R_(d12, r3, 0) NC_R_(d13, r3, 1088) NC_R_(d14, r3, 2112) NC_R_(d15, r3, 3200)
      "s_waitcnt lgkmcnt(0)"
      : [d0] "=&v"(d0), [d1] "=&v"(d1), [d2] "=&v"(d2), [d3] "=&v"(d3), [d4] "=&v"(d4), [d5] "=&v"(d5),
        [d6] "=&v"(d6), [d7] "=&v"(d7), [d8] "=&v"(d8), [d9] "=&v"(d9), [d10] "=&v"(d10), [d11] "=&v"(d11),
        [d12] "=&v"(d12), [d13] "=&v"(d13), [d14] "=&v"(d14), [d15] "=&v"(d15)
      : [wb] "v"(wb), [r0] "v"(r0), [r1] "v"(r1), [r2] "v"(r2), [r3] "v"(r3), [i0] "v"(i0), [i1] "v"(i1),
        [i2] "v"(i2), [i3] "v"(i3), [i4] "v"(i4), [i5] "v"(i5), [i6] "v"(i6), [i7] "v"(i7), [i8] "v"(i8),
        [i9] "v"(i9), [i10] "v"(i10), [i11] "v"(i11), [i12] "v"(i12), [i13] "v"(i13), [i14] "v"(i14),
        [i15] "v"(i15)
      : "memory");
  const nc_f2v d[16] = {d0, d1, d2, d3, d4, d5, d6, d7, d8, d9, d10, d11, d12, d13, d14, d15};
#pragma unroll
  for (int r = 0; r < 16; ++r) o[r] = make_float2(d[r].x, d[r].y);
}
#undef NC_W_
#undef NC_R_

// H512: hop 512 (the window path), whose hop slice [1024, 1536) of the frame is exactly stage-1
// rows r = 8..11 of every lane: the energy needs no per-sample membership test.  With the lane's
// Hann taps held in registers across frames (124 VGPRs, still four waves per SIMD) instead of 16
// LDS reads per frame: 483.3 -> 472.6 us per 560 windows, bit-identical (round 5,
// profiles/r5_stft_variants.txt; either change alone 483.8 / 479.1)
// EN: the f64 hop-slice energy of each frame (a.frame_energy); without it the window energies come
// from the silence trim's 512-sample block sums (nc_window_energy_blocks)
template <bool H512, bool EN, int J0 = kMelJ0, int J1 = kMelJ1>
__global__ __launch_bounds__(SM_THREADS) void stft_mel_kernel(StftMelArgs a) {
  const Span span_(a.span);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float2* sh_tw = reinterpret_cast<float2*>(smem);
  float4* sh_w4 = reinterpret_cast<float4*>(sh_tw + al4(SmTw::size));  // [mel_j0 + mel_j1][64]
  const int lane0 = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform (SGPR)
  float2* sh_hann = reinterpret_cast<float2*>(sh_w4 + (a.mel_j0 + a.mel_j1) * 64);
  int* sh_mt = reinterpret_cast<int*>(sh_hann + SM_HANN2);
  float2* slot = reinterpret_cast<float2*>(sh_mt + SM_MT) + wave * SM_HALF;

  __shared__ int sh_next;  // SM_DYN_: the workgroup's next frame
  if (threadIdx.x == 0) sh_next = 0;
  fill_staged_tw<1024>(sh_tw, a.tw, threadIdx.x, SM_THREADS);
  for (int i = threadIdx.x; i < SM_HANN2; i += SM_THREADS) sh_hann[i] = reinterpret_cast<const float2*>(a.hann2048)[i];
  for (int i = threadIdx.x; i < (a.mel_j0 + a.mel_j1) * 64; i += SM_THREADS) sh_w4[i] = a.mel_w4[i];
  if (threadIdx.x < SM_MT) sh_mt[threadIdx.x] = mel_pack(a.mel_lo4[threadIdx.x], a.mel_nj4[threadIdx.x], a.mel_band[threadIdx.x]);
  const float4* mw4 = sh_w4;
  // the slot zeroed once.  The mel steps past a band's end read slot floats [1025, mel_reach)
  // times a zero weight: until the first frame they hold these zeros, afterwards the frame's
  // own exchange-1/2 intermediates (the half-size exchanges write up to float 1055).  fmaf(0,
  // x, acc) == acc for every finite x, so the dB rows do not depend on them; an intermediate
  // overflowing to Inf would make a NaN there, but such a frame's power is Inf already
  for (int i = threadIdx.x & 63; i < SM_HALF; i += 64) slot[i] = make_float2(0.f, 0.f);
  __syncthreads();

  const int64_t n_groups = (a.total_frames + SM_WAVES - 1) / SM_WAVES;
  const int64_t gb = n_groups * blockIdx.x / gridDim.x, ge = n_groups * (blockIdx.x + 1) / gridDim.x;
  float2 hw[16];  // this lane's Hann taps, w[2 (j1 + 64 r)] and w[2 (j1 + 64 r) + 1]
  lds_read16_strided<0, 64 * 8>(hw, lds_addr(sh_hann + sm_j1(lane0)));
  // the wave's frames g = grp * SM_WAVES + wave rise by SM_WAVES: their sequence is tracked
  // forward, its bounds, flags, length and offset reloaded only when g crosses into a later
  // sequence, instead of a 64-bit division or binary search and dependent loads per frame.
  // (The workgroups keep static, balanced frame ranges: a chip-wide counter handing each wave runs
  // of N contiguous frames measured 4.64 (N = 128) and 11.5 (N = 512) against 3.42 ms per step
  // isolated — runs leave waves idle and break the CU's shared frame overlap,
  // profiles/r6_ab_summary.txt.  Inside a workgroup the frames are handed out one at a time.)
  int s = -1;
  int64_t sb = 0, se = -1, t0 = 0, L = 0, off = 0;
  int wc = -1;
  bool act = true;
  // SM_DYN_: the workgroup's frames [f0, f1) one at a time from its LDS counter (WgFrameQueue)
  const int64_t f0 = gb * SM_WAVES, f1 = std::min<int64_t>(ge * SM_WAVES, a.total_frames);
  WgFrameQueue fq(&sh_next, lane0);
  for (int64_t grp = gb; SM_DYN_ || grp < ge; ++grp) {
    int64_t g;
    if (SM_DYN_) {
      g = f0 + fq.take(lane0);
      if (g >= f1) break;
    } else {
      // (the probe's barrier orders nothing in memory: a bare s_barrier, no vmcnt / lgkmcnt drain)
      if (SM_SYNC_ > 0 && (grp - gb) % (SM_SYNC_ > 0 ? SM_SYNC_ : 1) == 0) __builtin_amdgcn_s_barrier();
      g = grp * SM_WAVES + wave;
      if (g >= a.total_frames) break;
    }
    if (g >= se) {
      if (s < 0) {
        s = a.frame_base ? seq_of_frame(a.frame_base, a.n_seq, g) : (int)(g / a.uniform_T);
      } else if (a.frame_base) {
        do ++s;
        while (s + 1 < a.n_seq && a.frame_base[s + 1] <= g);
      } else {
        s = (int)(g / a.uniform_T);
      }
      s = uniform32(s);
      sb = uniform64(a.frame_base ? a.frame_base[s] : (int64_t)s * a.uniform_T);
      se = uniform64(a.frame_base ? (s + 1 < a.n_seq ? a.frame_base[s + 1] : INT64_MAX) : sb + a.uniform_T);
      t0 = uniform64(a.frame_base && a.seq_t0 ? a.seq_t0[s] : 0);
      act = !a.active || a.active[s];
      L = uniform64(a.seq_len ? a.seq_len[s] : a.uniform_len);
      off = uniform64(a.seq_off[s]);
      wc = uniform32(a.win_chunk ? a.win_chunk[s] : -1);
    }
    if (!act) continue;
    const int64_t t = g - sb + t0;
    const float* x = a.sig + off;
    const int64_t s0 = t * a.hop - 1024;

    int lane = lane0;
    asm volatile("" : "+v"(lane));
    const int jin = sm_j1(lane);  // this lane's stage-1 butterfly: samples x[2 (jin + 64 r)]
    const float2* twl = sh_tw;
    const float* hann = a.hann2048;
    float2 in[16];
    double e = 0.0;
    const bool interior = s0 >= 0 && s0 + 2048 <= L;
    if (interior) {
      float2 xv[16];
      if ((off & 1) == 0) {
        const float2* x2 = reinterpret_cast<const float2*>(x + s0);
#pragma unroll
        for (int r = 0; r < 16; ++r) xv[r] = x2[jin + 64 * r];
      } else {
        const float* xs = x + s0;
#pragma unroll
        for (int r = 0; r < 16; ++r) xv[r] = make_float2(xs[2 * (jin + 64 * r)], xs[2 * (jin + 64 * r) + 1]);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int n = jin + 64 * r;
        const float2 v = xv[r];
        const float2 h = hw[r];
        if (EN && r >= 8 && r < 12) {
          const bool in_hop = H512 || 2 * n - 1024 < a.hop;
          const double dx = in_hop ? (double)v.x : 0.0, dy = in_hop ? (double)v.y : 0.0;
          e = fma(dx, dx, e);
          e = fma(dy, dy, e);
        }
        in[r] = make_float2(v.x * h.x, v.y * h.y);
      }
    } else {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int n = jin + 64 * r;
        const int64_t i0 = s0 + 2 * n;
        const float x0 = (i0 >= 0 && i0 < L) ? x[i0] : 0.0f;
        const float x1 = (i0 + 1 >= 0 && i0 + 1 < L) ? x[i0 + 1] : 0.0f;
        if (EN && r >= 8 && r < 12) {
          const int q = 2 * n - 1024;
          if (q < a.hop) {
            e = fma((double)x0, (double)x0, e);
            e = fma((double)x1, (double)x1, e);
          }
        }
        in[r] = make_float2(x0 * hann[2 * n], x1 * hann[2 * n + 1]);
      }
    }
    if (EN) {
      e = wave_sum_u(e);
      if (lane == 0) a.frame_energy[g] = e;
    }
    // stage 1 in registers, exchange 1, stage 2 (stockham_stage<1024, 16, 16, ...>'s twiddles and
    // DFT), exchange 2, the mirror-paired last stage
    DFT<16>::run(in);
    const int j2 = sm_j2(lane), k2 = j2 & 15;
    float2 v2[16];
    sm_exchange1(in, v2, lds_addr(slot + 8 * jin + (jin >> 2)), lds_addr(slot + (lane & 31)));
    {
      const uint32_t ta = lds_addr(twl + k2);
      tw_batch3<0, 16 * 8>(v2 + 1, ta);
      tw_batch3<3, 16 * 8>(v2 + 4, ta);
      tw_batch3<6, 16 * 8>(v2 + 7, ta);
      tw_batch3<9, 16 * 8>(v2 + 10, ta);
      tw_batch3<12, 16 * 8>(v2 + 13, ta);
    }
    DFT<16>::run(v2);
    float2 v[4][4];
    {
      const int b2 = j2 >> 4;
      float2 o[16];
      sm_exchange2(v2, o, lds_addr(slot + sm_boff(b2) + k2), lds_addr(slot + mirror_J(lane, 0)),
                   lds_addr(slot + mirror_J(lane, 1)), lds_addr(slot + (mirror_J(lane, 2) - 128)),
                   lds_addr(slot + (mirror_J(lane, 3) - 128)));
      static_for<4>([&](auto bc) {
        constexpr int b = decltype(bc)::value;
        float2 w[3];
        const uint32_t ta = lds_addr(twl + SmTw::s3 + mirror_J(lane, b));
        lds_read3<0, 2048, 4096>(w, ta, ta, ta);
        v[b][0] = o[4 * b];
#pragma unroll
        for (int r = 1; r < 4; ++r) v[b][r] = cmul(o[4 * b + r], w[r - 1]);
        DFT<4>::run(v[b]);
      });
    }
    // power |2 X[k]|^2 = 4 P[k], k in [0, 1024], over the slot (the split without its 0.5
    // scalings, exact; the mel weights carry the 0.25); a shared tuning frame (a leading frame of
    // a window that starts a 20 s chunk) also keeps its frame max for piptrack
    float* pw = reinterpret_cast<float*>(slot);
    const bool pip = wc >= 0 && t < a.tp_frames;
    float pmax = 0.0f;
    if (pip) {
      rsplit_mirror<SmTw::split, false>(v, twl, lane, [&](int k, float2 X, float2 XN) {
        const float p1 = fmaf(X.x, X.x, X.y * X.y), p2 = fmaf(XN.x, XN.x, XN.y * XN.y);
        pw[k] = p1;
        pw[1024 - k] = p2;
        pmax = fmaxf(pmax, fmaxf(p1, p2));
      });
    } else {
      rsplit_mirror<SmTw::split, false>(v, twl, lane, [&](int k, float2 X, float2 XN) {
        pw[k] = fmaf(X.x, X.x, X.y * X.y);
        pw[1024 - k] = fmaf(XN.x, XN.x, XN.y * XN.y);
      });
    }
    // Slaney mel: lane l owns one short and one long band (mel_band: spread over the lanes so
    // the float4 power reads are bank-conflict free), read as float4 steps from a 16-byte
    // aligned first bin with zero-padded weights (fmaf chain in bin order, as the CSR form)
    float acc0 = 0.0f, acc1 = 0.0f;
    const int mt0 = sh_mt[lane], mt1 = sh_mt[64 + lane];
    mel_unrolled<J0>(pw, mw4, mt0 & 2047, (mt0 >> 11) & 31, lane, acc0);
    mel_unrolled<J1>(pw, mw4 + J0 * 64, mt1 & 2047, (mt1 >> 11) & 31, lane, acc1);
    const float db0 = db10_floor(acc0);  // = 10 log10f(max(1e-10, acc0)), bit for bit
    const float db1 = db10_floor(acc1);
    float* row = a.sdb + g * 128;
    row[mt0 >> 16] = db0;
    row[mt1 >> 16] = db1;
    const float mx = wave_max_u(fmaxf(db0, db1));
    if (lane == 0) a.frame_max[g] = mx;
    if (pip) {
      // estimate_tuning's piptrack on the same 2|X| values tuning_peaks_kernel computes
      // (nc_piptrack.h): |X| of the stencil bins written over the power in place (bin k at
      // float k - (kPipLo - 1)).  A lane's store of round q + 1 hits bins that other lanes read
      // in round q, and per-lane alias analysis lets the compiler order them either way, so
      // every round's power is read into registers first, and the stores follow a compiler
      // barrier (one wave's LDS operations then complete in program order)
      const float pm = __fsqrt_rn(wave_max_u(pmax));
      constexpr int kPipQ = (kPipHi - kPipLo + 3 + 63) / 64;
      float pv[kPipQ];
#pragma unroll
      for (int q = 0; q < kPipQ; ++q) {
        const int k = kPipLo - 1 + 64 * q + lane;
        pv[q] = (64 * (q + 1) <= kPipHi - kPipLo + 3 || k <= kPipHi + 1) ? pw[k] : 0.0f;
      }
      asm volatile("" ::: "memory");
#pragma unroll
      for (int q = 0; q < kPipQ; ++q) {
        const int k = kPipLo - 1 + 64 * q + lane;
        if (64 * (q + 1) <= kPipHi - kPipLo + 3 || k <= kPipHi + 1) pw[k - (kPipLo - 1)] = __fsqrt_rn(pv[q]);
      }
      const int64_t base = uniform64(a.chunk_tf_base[wc]) * kPeakSlots;
      piptrack_append([&](int k) { return pw[k - (kPipLo - 1)]; }, pm, lane, &a.chunk_npk[wc], a.peak_pitch + base,
                      a.peak_mag + base, reinterpret_cast<int*>(pw + kPipKpkHalf));
    }
  }
}

int launch_stft_mel(Context& ctx, const StftMelArgs& args, hipStream_t st) {
  if (args.total_frames <= 0) return 0;
  StftMelArgs a = args;
  a.tw = ctx.t.tw;
  a.hann2048 = ctx.t.hann2048;
  a.mel_lo = ctx.t.mel_lo;
  a.mel_len = ctx.t.mel_len;
  a.mel_off = ctx.t.mel_off;
  a.mel_w = ctx.t.mel_w;
  a.mel_nnz = ctx.t.mel_nnz;
  a.mel_w4 = ctx.t.mel_w4;
  a.mel_lo4 = ctx.t.mel_lo4;
  a.mel_nj4 = ctx.t.mel_nj4;
  a.mel_band = ctx.t.mel_band;
  a.mel_j0 = ctx.t.mel_j0;
  a.mel_j1 = ctx.t.mel_j1;
  if (a.hop <= 0 || a.hop > 512 || (a.hop & 1)) {
    set_error("stft_mel: hop must be even and <= 512");
    return -2;
  }
  const bool wide = a.mel_j0 == kMelJ0w && a.mel_j1 == kMelJ1w;
  if (!(a.mel_j0 == kMelJ0 && a.mel_j1 == kMelJ1) && !wide) {
    set_error("stft_mel: mel table trip counts differ from the kernel's compile-time ones");
    return -2;
  }
  if (a.chunk_tf_base && ctx.sr != kSR) {
    set_error("stft_mel: the shared tuning frames (piptrack) are built for 22050 Hz");
    return -2;
  }
  const size_t lds = std::max<size_t>(stft_mel_lds_bytes(a.mel_j0 + a.mel_j1), SM_LDS_RESERVE);
  if (lds > 160 * 1024) {
    set_error("stft_mel: LDS layout exceeds 160 KiB");
    return -2;
  }
  if (ctx.t.mel_reach > 2 * SM_HALF) {
    set_error("stft_mel: the mel steps read past the half-size slot");
    return -2;
  }
  const int64_t n_groups = (a.total_frames + SM_WAVES - 1) / SM_WAVES;
  const int cus = ctx.stft_cus > 0 ? ctx.stft_cus : ctx.num_cu;
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(n_groups, (int64_t)cus * (lds <= 80 * 1024 ? 2 : 1)));
  {
    KTimer kt_(ctx, "stft_mel", st);
    a.span = kt_.span();
    const bool en = a.frame_energy != nullptr && !SM_NOEN_;
    if (wide) {  // a context at another sample rate (nc_create_rate): tempo seams only
      if (a.hop == 512 && en)
        hipLaunchKernelGGL((stft_mel_kernel<true, true, kMelJ0w, kMelJ1w>), dim3(grid), dim3(SM_THREADS), lds, st, a);
      else if (a.hop == 512)
        hipLaunchKernelGGL((stft_mel_kernel<true, false, kMelJ0w, kMelJ1w>), dim3(grid), dim3(SM_THREADS), lds, st, a);
      else if (en)
        hipLaunchKernelGGL((stft_mel_kernel<false, true, kMelJ0w, kMelJ1w>), dim3(grid), dim3(SM_THREADS), lds, st, a);
      else
        hipLaunchKernelGGL((stft_mel_kernel<false, false, kMelJ0w, kMelJ1w>), dim3(grid), dim3(SM_THREADS), lds, st, a);
    } else if (a.hop == 512 && en)
      hipLaunchKernelGGL((stft_mel_kernel<true, true>), dim3(grid), dim3(SM_THREADS), lds, st, a);
    else if (a.hop == 512)
      hipLaunchKernelGGL((stft_mel_kernel<true, false>), dim3(grid), dim3(SM_THREADS), lds, st, a);
    else if (en)
      hipLaunchKernelGGL((stft_mel_kernel<false, true>), dim3(grid), dim3(SM_THREADS), lds, st, a);
    else
      hipLaunchKernelGGL((stft_mel_kernel<false, false>), dim3(grid), dim3(SM_THREADS), lds, st, a);
  }
  NC_HIP(hipGetLastError());
  return 0;
}

}  // namespace nc
