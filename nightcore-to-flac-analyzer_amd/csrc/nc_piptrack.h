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

// One wave, one frame.  mag(k) = |X[k]| (k in [kPipLo - 1, kPipHi + 1]), mx = max_k |X[k]|
// over all 1025 bins.  Peaks are appended to the chunk's list at an atomically reserved
// position (its consumers, median and histogram, do not depend on the order).
template <class Mag>
__device__ __forceinline__ void piptrack_append(Mag&& mag, float mx, int lane, int* npk, float* pp, float* pm) {
  const float ref = 0.1f * mx;
  float pitch[kPipRounds], pmag[kPipRounds];
  unsigned long long bal[kPipRounds];
  int cnt = 0;
#pragma unroll
  for (int q = 0; q < kPipRounds; ++q) {
    const int k = kPipLo + 64 * q + lane;
    bool pk = false;
    pitch[q] = 0.0f;
    pmag[q] = 0.0f;
    if (k <= kPipHi) {
      const float sm = mag(k - 1), s = mag(k), sp = mag(k + 1);
      const float zm = sm > ref ? sm : 0.0f, z = s > ref ? s : 0.0f, zp = sp > ref ? sp : 0.0f;
      pk = (z > zm) && (z >= zp);
      if (pk) {
        // parabolic shift (librosa numba stencil, f64 arithmetic, stored f32)
        const double aa = (double)(sp + sm) - 2.0 * (double)s;  // f32 add, then f64 (numba typing)
        const double bb = (double)(sp - sm) / 2.0;
        const float shift = (fabs(bb) >= fabs(aa)) ? 0.0f : (float)(-bb / aa);
        const float avg = (sp - sm) / 2.0f;
        const float dskew = (0.5f * avg) * shift;
        pitch[q] = (float)((((double)k + (double)shift) * 22050.0) / 2048.0);
        pmag[q] = s + dskew;
      }
    }
    bal[q] = __ballot(pk);
    cnt += __popcll(bal[q]);
  }
  if (cnt == 0) return;
  int pos = 0;
  if (lane == 0) pos = atomicAdd(npk, cnt);
  pos = __shfl(pos, 0, 64);
  const unsigned long long below = (1ull << lane) - 1ull;
#pragma unroll
  for (int q = 0; q < kPipRounds; ++q) {
    if ((bal[q] >> lane) & 1ull) {
      const int i = pos + __popcll(bal[q] & below);
      pp[i] = pitch[q];
      pm[i] = pmag[q];
    }
    pos += __popcll(bal[q]);
  }
}

}  // namespace nc
