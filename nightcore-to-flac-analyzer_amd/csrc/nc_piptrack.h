// nc_piptrack.h — the piptrack peak stencil of librosa.estimate_tuning (n_fft 2048,
// fmin 150, fmax 4000, threshold 0.1 of the frame's max |X|; oracle/ncref.py piptrack),
// shared by tuning_peaks_kernel (cqt.hip, every tuning frame of a chunk) and
// stft_mel_kernel (stft.hip, the leading tuning frames that coincide with a window's own
// STFT frames), so that both produce bit-identical peaks.
#pragma once
#include "nc_device.h"

namespace nc {

constexpr int kPeakSlots = 192;     // >= max piptrack peaks per frame (bins 14..371 -> <= 179)
constexpr int kPipLo = 14, kPipHi = 371;  // [150, 4000) Hz at sr 22050, n_fft 2048: k 22050 / 2048
constexpr int kPipRounds = (kPipHi - kPipLo + 64) / 64;
// Float offsets inside a wave's 1024-point FFT slot (LdsSize<1024> = 2112 floats) past the
// power spectrum [0, 1025): |X| of the stencil bins kPipLo - 1 .. kPipHi + 1 (stft_mel keeps
// the power intact for the mel step) and the compacted peak bins.
constexpr int kPipMag = 1088, kPipKpk = 1472;
static_assert(kPipMag >= 1025 && kPipMag + (kPipHi - kPipLo + 3) <= kPipKpk, "piptrack slot layout");
static_assert(kPipKpk + (kPipHi - kPipLo + 1) <= 2112, "piptrack slot layout");
static_assert(kPipHi + 1 < 512, "tuning_peaks stores only the split's low half (bins <= 512)");

// One wave, one frame.  mag(k) = |X[k]| (k in [kPipLo - 1, kPipHi + 1]), mx = max_k |X[k]|
// over all 1025 bins.  Peaks are appended to the chunk's list at an atomically reserved
// position (its consumers, median and histogram, do not depend on the order).
// The stencil decision runs bin-parallel (6 rounds of 64 bins); the peaks' bins are compacted
// through kpk (wave-private LDS, >= kPipHi - kPipLo + 1 ints) so the f64 parabolic shift and
// the list stores run once per 64 peaks (about 10 per frame) instead of once per round under
// a divergent mask.  Same list positions (round-major, lane order) and values as the
// per-round form.
template <class Mag>
__device__ __forceinline__ void piptrack_append(Mag&& mag, float mx, int lane, int* npk, float* pp, float* pm,
                                                int* kpk) {
  const float ref = 0.1f * mx;
  const unsigned long long below = (1ull << lane) - 1ull;
  int cnt = 0;
#pragma unroll
  for (int q = 0; q < kPipRounds; ++q) {
    const int k = kPipLo + 64 * q + lane;
    bool pk = false;
    if (64 * (q + 1) <= kPipHi - kPipLo + 1 || k <= kPipHi) {  // only the last round is partial
      const float sm = mag(k - 1), s = mag(k), sp = mag(k + 1);
      const float zm = sm > ref ? sm : 0.0f, z = s > ref ? s : 0.0f, zp = sp > ref ? sp : 0.0f;
      pk = (z > zm) && (z >= zp);
    }
    const unsigned long long bal = __ballot(pk);
    if (pk) kpk[cnt + __popcll(bal & below)] = k;
    cnt += __popcll(bal);
  }
  cnt = __builtin_amdgcn_readfirstlane(cnt);
  if (cnt == 0) return;
  int pos = 0;
  if (lane == 0) pos = atomicAdd(npk, cnt);
  pos = __builtin_amdgcn_readfirstlane(__shfl(pos, 0, 64));
  for (int j = lane; j - lane < cnt; j += 64) {
    if (j < cnt) {
      const int k = kpk[j];
      const float sm = mag(k - 1), s = mag(k), sp = mag(k + 1);
      // parabolic shift (librosa numba stencil, f64 arithmetic, stored f32)
      const double aa = (double)(sp + sm) - 2.0 * (double)s;  // f32 add, then f64 (numba typing)
      const double bb = (double)(sp - sm) / 2.0;
      const float shift = (fabs(bb) >= fabs(aa)) ? 0.0f : (float)(-bb / aa);
      const float avg = (sp - sm) / 2.0f;
      const float dskew = (0.5f * avg) * shift;
      pp[pos + j] = (float)((((double)k + (double)shift) * 22050.0) / 2048.0);
      pm[pos + j] = s + dskew;
    }
  }
}

}  // namespace nc
