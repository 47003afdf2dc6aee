// stft_args.h — argument block of stft_mel_kernel (stft.hip), shared with its callers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nc {

struct Context;

struct StftMelArgs {
  const float* sig;
  const int64_t* seq_off;     // [n_seq] sample offsets into sig
  const int64_t* seq_len;     // [n_seq] or nullptr: every sequence is uniform_len long
  const int64_t* frame_base;  // [n_seq + 1] or nullptr: every sequence has uniform_T frames
  const int64_t* seq_t0 = nullptr;  // nullable [n_seq]: frame g of sequence s is its STFT frame
                                    // seq_t0[s] + (g - frame_base[s]) (a frame range of a file)
  int64_t uniform_len;
  int uniform_T;
  int n_seq;
  int64_t total_frames;
  const uint8_t* active;  // nullable: frames of sequences with active[s] == 0 are skipped
  int hop;
  float* sdb;             // [total_frames][128]
  float* frame_max;       // [total_frames]
  double* frame_energy;   // nullable [total_frames]: sum x^2 over [t hop, (t+1) hop) of the sequence
  const float2* tw;       // global 8192-entry table
  const float* hann2048;
  const int* mel_lo;
  const int* mel_len;
  const int* mel_off;
  const float* mel_w;
  int mel_nnz;
  const float4* mel_w4;
  const int* mel_lo4;
  const int* mel_nj4;
  const int* mel_band;
  int mel_j0, mel_j1;
  // shared tuning frames (nullable win_chunk): frames t < tp_frames of sequence s with
  // win_chunk[s] = c >= 0 are also tuning frames t of chunk c; their piptrack peaks are
  // appended to chunk c's list (peak_*[chunk_tf_base[c] * kPeakSlots ..], count chunk_npk[c])
  const int* win_chunk;
  const int64_t* chunk_tf_base;
  int tp_frames;
  float* peak_pitch;
  float* peak_mag;
  int* chunk_npk;
  unsigned long long* span = nullptr;  // nc_profile execution span (nc_device.h)
};

int launch_stft_mel(Context& ctx, const StftMelArgs& args, hipStream_t st);

}  // namespace nc
