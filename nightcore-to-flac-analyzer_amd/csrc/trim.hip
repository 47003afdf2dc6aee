// trim.hip — K1a: librosa.effects.trim(y, top_db) as called by io.strip_silence
// (io.py:58-79).  oracle: ncref.trim / ncref.rms_frames.
//
//   ms[t]   = mean_{2048-sample centred frame t, zero padded} x^2     (hop 512)
//   rms[t]  = sqrt(ms[t]) (f32);  db[t] = 10 log10(max(1e-10, rms^2)) - 10 log10(max(1e-10, max(rms)^2))
//   start   = first(db > -top_db) * 512,  end = min(N, (last + 1) * 512)
//
// Kernel 1: f64 sums of x^2 over 512-sample blocks (one wave per block, each sample
// read once from HBM); kernel 2: one workgroup per file forms each frame's mean
// from its 4 blocks, then the max and the first/last frames above -top_db.
#include "nc_block.h"
#include "nc_engine.h"

namespace nc {

// f64 sum of x^2 over each 512-sample block b = [512 b, 512 b + 512) of each file, every
// sample read once; block b of file f at blk[frame_base[f] + b].  One workgroup per tile of
// TR_BPG blocks of one file (tile_base[f] = first tile of file f: one search per workgroup,
// not per wave); each wave sums TR_BPW consecutive blocks with all their 16-byte loads in flight.
#ifndef TR_BSEARCH
#define TR_BSEARCH 0
#endif
constexpr int TR_BPW = 4;                  // blocks per wave
constexpr int TR_BPG = 4 * TR_BPW;         // blocks per workgroup (4 waves)

__global__ __launch_bounds__(256) void trim_blocks_kernel(const float* sig, const int64_t* file_off,
                                                          const int64_t* file_len, const int64_t* frame_base,
                                                          const int64_t* tile_base, int n_files, double* blk,
                                                          unsigned long long* span) {
  const Span span_(span);
  const int lane = threadIdx.x & 63;
  const int64_t tile = blockIdx.x;
  // the tile's file = the last f with tile_base[f] <= tile (tile_base is non-decreasing): the
  // wave counts the entries <= tile, 64 independent loads per round, instead of a binary
  // search's chain of dependent scalar loads (7 round trips for 116 files) ahead of every
  // workgroup's sample loads.  Entry n_files (the tile total) counts too: past it, no tile.
#if TR_BSEARCH  // the round-3 binary search (A/B builds only)
  if (tile >= tile_base[n_files]) return;
  int lo = 0, hi = n_files - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (tile_base[mid] <= tile) lo = mid;
    else hi = mid - 1;
  }
  const int f = __builtin_amdgcn_readfirstlane(lo);
#else
  int cnt = 0;
  for (int i0 = 0; i0 <= n_files; i0 += 64) {
    const int i = i0 + lane;
    cnt += __popcll(__ballot(i <= n_files && tile_base[i] <= tile));
  }
  if (cnt > n_files) return;
  const int f = __builtin_amdgcn_readfirstlane(cnt - 1);
#endif
  const int64_t N = file_len[f];
  const int64_t nblk = (N + 511) / 512;
  const int64_t b0 = (tile - tile_base[f]) * TR_BPG + (threadIdx.x >> 6) * TR_BPW;
  if (b0 >= nblk) return;
  const int64_t off = file_off[f];
  double acc[TR_BPW];
  if ((b0 + TR_BPW) * 512 <= N && ((off + b0 * 512) & 3) == 0) {
    const float4* x4 = reinterpret_cast<const float4*>(sig + off + b0 * 512);
    float4 v[TR_BPW][2];
#pragma unroll
    for (int i = 0; i < TR_BPW; ++i)
#pragma unroll
      for (int q = 0; q < 2; ++q) v[i][q] = x4[i * 128 + lane + 64 * q];
#pragma unroll
    for (int i = 0; i < TR_BPW; ++i) {
      double a = 0.0;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        a = fma((double)v[i][q].x, (double)v[i][q].x, a);
        a = fma((double)v[i][q].y, (double)v[i][q].y, a);
        a = fma((double)v[i][q].z, (double)v[i][q].z, a);
        a = fma((double)v[i][q].w, (double)v[i][q].w, a);
      }
      acc[i] = a;
    }
  } else {
    const float* x = sig + off;
#pragma unroll
    for (int i = 0; i < TR_BPW; ++i) {
      double a = 0.0;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int64_t j = (b0 + i) * 512 + lane + 64 * q;
        const double v = j < N ? (double)x[j] : 0.0;
        a = fma(v, v, a);
      }
      acc[i] = a;
    }
  }
#pragma unroll
  for (int i = 0; i < TR_BPW; ++i) {
    const double a = wave_sum(acc[i]);
    if (lane == 0 && b0 + i < nblk) blk[frame_base[f] + b0 + i] = a;
  }
}

// ms[t] = mean of x^2 over the centred 2048-sample frame t = blocks t-2 .. t+1 (zero outside)
__device__ __forceinline__ float trim_ms(const double* blk, int64_t nblk, int64_t t) {
  double s = 0.0;
#pragma unroll
  for (int d = -2; d <= 1; ++d) {
    const int64_t b = t + d;
    if (b >= 0 && b < nblk) s += blk[b];
  }
  return (float)(s / 2048.0);
}

__global__ __launch_bounds__(256) void trim_bounds_kernel(const double* blk_all, const int64_t* frame_base,
                                                          const int64_t* file_len, float top_db,
                                                          int64_t* out_start, int64_t* out_end) {
  __shared__ BlockScratch<256> bs;
  const int f = blockIdx.x;
  const int64_t N = file_len[f];
  const int64_t T = 1 + N / 512;
  const int64_t nblk = (N + 511) / 512;
  const double* blk = blk_all + frame_base[f];
  double mx = -1.0;
  for (int64_t t = threadIdx.x; t < T; t += 256) mx = fmax(mx, (double)sqrtf(trim_ms(blk, nblk, t)));
  mx = block_max<256>(mx, bs);
  const float ref = (float)mx;
  const float ref_db = 10.0f * log10f(fmaxf(1e-10f, ref * ref));
  int first = 0x7fffffff, last = -1;
  for (int64_t t = threadIdx.x; t < T; t += 256) {
    const float r = sqrtf(trim_ms(blk, nblk, t));
    const float db = 10.0f * log10f(fmaxf(1e-10f, r * r)) - ref_db;
    if (db > -top_db) {
      first = min(first, (int)t);
      last = max(last, (int)t);
    }
  }
  first = block_min_i<256>(first, bs);
  last = block_max_i<256>(last, bs);
  if (threadIdx.x == 0) {
    if (last >= 0) {
      out_start[f] = (int64_t)first * 512;
      out_end[f] = min(N, ((int64_t)last + 1) * 512);
    } else {
      out_start[f] = 0;
      out_end[f] = 0;
    }
  }
}

size_t trim_ws_bytes(const int64_t* host_file_len, int n_files) {
  size_t frames = 0;
  for (int f = 0; f < n_files; ++f) frames += 1 + host_file_len[f] / 512;
  return frames * sizeof(double) + 2 * (size_t)(n_files + 1) * sizeof(int64_t) + 256;
}

// frame_base is computed on the device from file_len (parallel exclusive scan, one block)
__global__ __launch_bounds__(256) void frame_base_kernel(const int64_t* file_len, int n_files, int64_t* frame_base,
                                                         int64_t* tile_base) {
  block_prefix_table<256>(n_files, frame_base, [&](int f) { return 1 + file_len[f] / 512; });
  block_prefix_table<256>(n_files, tile_base,
                          [&](int f) { return ((file_len[f] + 511) / 512 + TR_BPG - 1) / TR_BPG; });
}

int launch_trim(Context& ctx, const float* sig, const int64_t* file_off, const int64_t* file_len, int n_files,
                int64_t max_frames, float top_db, int64_t* out_start, int64_t* out_end, void* ws,
                size_t ws_bytes, hipStream_t st) {
  (void)ctx;
  if (n_files <= 0) return 0;
  // max_frames = total frames over all files (host knows the lengths)
  const size_t need = (size_t)max_frames * sizeof(double) + 2 * (size_t)(n_files + 1) * sizeof(int64_t);
  if (ws_bytes < need) {
    set_error("trim: workspace too small");
    return -3;
  }
  int64_t* frame_base = static_cast<int64_t*>(ws);
  int64_t* tile_base = frame_base + n_files + 1;
  double* blk = reinterpret_cast<double*>(tile_base + n_files + 1);
  hipLaunchKernelGGL(frame_base_kernel, dim3(1), dim3(256), 0, st, file_len, n_files, frame_base, tile_base);
  // tiles <= sum over files of ceil(blocks / TR_BPG) <= max_frames / TR_BPG + n_files
  const int64_t tiles = max_frames / TR_BPG + n_files + 1;
  {
    KTimer kt_(ctx, "trim_blocks", st);
    hipLaunchKernelGGL(trim_blocks_kernel, dim3((unsigned)tiles), dim3(256), 0, st, sig, file_off, file_len,
                       frame_base, tile_base, n_files, blk, kt_.span());
  }
  {
    MarkSpan ms_(ctx, "trim_bounds", st);
    hipLaunchKernelGGL(trim_bounds_kernel, dim3(n_files), dim3(256), 0, st, blk, frame_base, file_len, top_db,
                       out_start, out_end);
  }
  NC_HIP(hipGetLastError());
  return 0;
}

// Window energies from the trim's block sums (io.slice_windows' energy_db, io.py:38-40):
//   E = sum over [s, s + L) of x^2,  s = win_off[w] - file_off[f],  f = win_file[w]
// the full 512-sample blocks of file f inside the window from blk (trim_blocks_kernel's f64 sums
// of exactly these samples), the partial blocks at either end from the samples themselves; one
// wave per window, each lane's f64 partials in a fixed order, then the wave sum (deterministic).
// energy_db = 20 log10(max(sqrt(E / L), 1e-10)).  stft_mel then needs no per-frame energy.
__global__ __launch_bounds__(256) void window_energy_blocks_kernel(const float* sig, const int64_t* trim_ws, int n_files,
                                                                   const int64_t* file_off, const int64_t* win_off,
                                                                   const int* win_file, int n_win, int L,
                                                                   double* out) {
  const int lane = threadIdx.x & 63;
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (w >= n_win) return;
  const int f = win_file[w];
  const int64_t* frame_base = trim_ws;
  const double* blk = reinterpret_cast<const double*>(trim_ws + 2 * (n_files + 1)) + frame_base[f];
  const int64_t fo = file_off[f];
  const int64_t s = win_off[w] - fo, e = s + L;
  int64_t b0 = (s + 511) / 512, b1 = e / 512;  // full blocks [b0, b1)
  if (b1 < b0) b1 = b0;
  const int64_t h1 = min(e, 512 * b0), t0 = max(h1, 512 * b1);  // head [s, h1), tail [t0, e)
  const float* x = sig + fo;
  double acc = 0.0;
  for (int64_t b = b0 + lane; b < b1; b += 64) acc += blk[b];
  for (int64_t i = s + lane; i < h1; i += 64) {
    const double v = (double)x[i];
    acc = fma(v, v, acc);
  }
  for (int64_t i = t0 + lane; i < e; i += 64) {
    const double v = (double)x[i];
    acc = fma(v, v, acc);
  }
  acc = wave_sum(acc);
  if (lane == 0) out[w] = 20.0 * log10(fmax(sqrt(acc / (double)L), 1e-10));
}

int launch_window_energy_blocks(const float* sig, const void* trim_ws, int n_files, const int64_t* file_off,
                                const int64_t* win_off, const int* win_file, int n_win, int win_len, double* out,
                                hipStream_t st) {
  if (n_win <= 0) return 0;
  if (n_files <= 0 || win_len <= 0) {
    set_error("window_energy_blocks: need trimmed files and a positive window length");
    return -2;
  }
  hipLaunchKernelGGL(window_energy_blocks_kernel, dim3((n_win + 3) / 4), dim3(256), 0, st, sig,
                     static_cast<const int64_t*>(trim_ws), n_files, file_off, win_off, win_file, n_win, win_len, out);
  NC_HIP(hipGetLastError());
  return 0;
}

}  // namespace nc
