/*
 * ncgpu.h — C ABI of the MI355X nightcore analysis engine (libncgpu.so).
 *
 * The drop-in boundary of this repository.  The reference
 * (Tealdragon204/nightcore-to-flac-analyzer) is pure Python and has no FFI; each
 * entry point below replaces the reference function (file:line under
 * nightcore_analyzer/) or the librosa call it makes on the hot path, and is
 * bound from Python by ctypes in nightcore-to-flac-analyzer_amd/nightcore_analyzer/_native.py
 * (the binding a maintainer would add is shown in INTEGRATION.md).
 *
 * Conventions
 *   - plain pointers and sizes only; every array pointer is DEVICE memory
 *     (hipMalloc / torch.cuda tensors) unless documented otherwise;
 *   - all work is stream-ordered on the `stream` argument (a hipStream_t; NULL =
 *     the default stream); no entry point synchronises or allocates except
 *     nc_create/nc_destroy, so a sequence of calls can be captured in a hipGraph;
 *   - scratch comes from a caller-owned workspace of `*_workspace_bytes` bytes;
 *   - every call returns 0 on success, < 0 on error; nc_last_error() returns a
 *     thread-local message for the last failure on the calling thread;
 *   - one context per (device, thread); contexts hold only read-only tables.
 *
 * Signals: mono float32 at 22 050 Hz, concatenated in one buffer; windows,
 * chunks and files are addressed by int64 sample offsets into it ("views", as
 * the reference's AudioWindow.audio is a numpy view, io.py:100).
 */
#ifndef NCGPU_H
#define NCGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct nc_ctx nc_ctx;

#define NCGPU_ABI_VERSION 1

int nc_abi_version(void);
const char* nc_last_error(void);

/* Create / destroy a context on `device` (builds the f32 constant tables:
 * twiddles, Hann windows, Slaney mel bank, CQT bases for the 100-value tuning
 * grid, the half-band decimator). */
int nc_create(int device, nc_ctx** out);
int nc_destroy(nc_ctx* ctx);
/* number of compute units seen by the context (256 on MI355X) */
int nc_num_cu(const nc_ctx* ctx);

/* ---------------------------------------------------------------------------
 * K1a  silence trim — replaces io.strip_silence (io.py:58-79) ->
 *      librosa.effects.trim(y, top_db) (io.py:76).
 * For each file f: samples [file_off[f], file_off[f]+file_len[f]) of `sig`;
 * frame RMS (2048/512, centred, zero pad) -> dB re max -> non-silent frames
 * (> -top_db) -> out_start[f] / out_end[f] (sample indices relative to the file,
 * start = first*512, end = min(len, (last+1)*512); 0/0 for an all-silent file).
 * ------------------------------------------------------------------------- */
size_t nc_trim_workspace_bytes(const int64_t* host_file_len, int n_files);
int nc_trim_bounds(nc_ctx* ctx, const float* sig, const int64_t* file_off, const int64_t* file_len,
                   int n_files, int64_t max_frames, float top_db, int64_t* out_start,
                   int64_t* out_end, void* ws, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * K1b+K2..K5  per-window stage — replaces io._rms_db (io.py:38-40) and, inside
 * tempo.estimate_tempo (tempo.py:27-77), librosa.onset.onset_strength
 * (tempo.py:44) and the tempogram mean behind beat_track/feature.tempo
 * (tempo.py:45-50, 61-68).
 * Window w = win_len samples at sig + win_off[w] (hop must be 512).
 * Outputs: onset_out[w*T + t] (T = 1 + win_len/512), tg_out[w*acw + k]
 * (acw = 344: mean over frames of the inf-normalised tempogram),
 * energy_out[w] (RMS dB, float64).  `active` (nullable) skips windows.
 * ------------------------------------------------------------------------- */
size_t nc_window_stage_workspace_bytes(const nc_ctx* ctx, int n_win, int win_len, int hop);
int nc_window_stage(nc_ctx* ctx, const float* sig, const int64_t* win_off, const uint8_t* active,
                    int n_win, int win_len, int hop, float* onset_out, double* tg_out,
                    double* energy_out, void* ws, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * K6..K8  tempo + beat tracking — replaces librosa.beat.beat_track(onset_envelope,
 * sr, hop_length, start_bpm) as called at tempo.py:45-50 (windows) and
 * tempo.py:159-164 (full signal); with feature.tempo (tempo.py:63) giving the
 * identical tempo, this is all of estimate_tempo after the onset envelope.
 * Sequence s: onset[off[s] .. off[s]+len[s]), tempogram mean tg[s*acw ..].
 * start_bpm: per sequence, or per group when prior_idx != NULL
 * (start = start_bpm[prior_idx[s]]).
 * Outputs: bpm_out (tempo, float64; 0 when the onset envelope is all zero),
 * lag_out (tempogram lag), nbeats_out (beats after trimming; -1 = capacity
 * error), margin_out (nullable: score gap to the runner-up lag),
 * beats_out (nullable: beat frames written at off[s]).
 * Workspace needed only when max_len is too long for LDS (hop-64 signals).
 * ------------------------------------------------------------------------- */
size_t nc_tempo_beats_workspace_bytes(int64_t total_frames);
int nc_tempo_beats(nc_ctx* ctx, const float* onset, const int64_t* off, const int* len, int n_seq,
                   int max_len, const double* tg, int acw, const double* start_bpm,
                   const int* prior_idx, const uint8_t* active, int hop, int trim, double* bpm_out,
                   int* lag_out, int* nbeats_out, double* margin_out, int* beats_out,
                   int64_t total_frames, void* ws, size_t ws_bytes, void* stream);

/* nc tempo prior — pipeline.py:174-183: median of the valid source-window
 * tempos (active and nbeats >= 4) of pair p (windows [src_w0[p], src_w1[p]))
 * times src_len[p]/nc_len[p]; 120 when none is valid. */
int nc_tempo_prior(nc_ctx* ctx, const double* bpm, const int* nbeats, const uint8_t* active,
                   const int* src_w0, const int* src_w1, const int64_t* src_len,
                   const int64_t* nc_len, int n_pairs, double* prior_out, void* stream);

/* tempo.py:165-172 — inter-beat intervals (s) of each beat list, glitches
 * (<= 0.05 s) removed; n_ibi[s] = 0 when fewer than min_ibis remain (None). */
int nc_ibi_from_beats(nc_ctx* ctx, const int* beats, const int64_t* off, const int* nbeats, int n_seq,
                      int hop, int min_ibis, double* ibi_out, int* n_ibi, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* NCGPU_H */
