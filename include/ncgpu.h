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

#define NCGPU_ABI_VERSION 5  /* 5: nc_pcm16_to_f32; 4: nc_melodia_salience; 3: tuning decision margins, nc_xcorr_peak */

int nc_abi_version(void);
const char* nc_last_error(void);

/* Create / destroy a context on `device` (builds the f32 constant tables:
 * twiddles, Hann windows, Slaney mel bank, CQT bases for the 100-value tuning
 * grid, the half-band decimator). */
int nc_create(int device, nc_ctx** out);
/* The same for audio at `sample_rate` Hz (ABI 5; 8000..48000): the mel bank and the tempogram
 * windows are built for that rate, so the per-window stage, the beat tracker and the hop-64 IBI
 * pass follow tempo.py:27-173 at that sr (librosa passes sr through).  The CQT / tuning tables
 * stay at 22 050 Hz: the chroma entry points and the shared tuning frames need nc_create. */
int nc_create_rate(int device, int sample_rate, nc_ctx** out);
int nc_destroy(nc_ctx* ctx);
/* number of compute units seen by the context (256 on MI355X) */
int nc_num_cu(const nc_ctx* ctx);

/* Opt-in per-kernel timing (no reference equivalent; measurement only).
 * on = 1: the dominant kernels are bracketed by HIP events on their stream AND record
 *         their own execution span; on = 2: spans only (no host work per launch, cheap
 *         enough for a timed region); on = 3: events only around the roofline kernels
 *         ("stft_mel", "cqt_low", "cqt_high", "window_tg"), spans for every kernel (the
 *         other kernels' event records are host and queue work a timed region need not
 *         carry); on = 4: the events of on = 3 without spans (the spans' per-workgroup clock
 *         reads and atomics cost the step ~3 %); on = 5: the spans of on = 2 plus marker
 *         spans around the small entry points (nc_energy_gate, nc_collect_valid, nc_pitch_hz,
 *         nc_tempo_prior, nc_bootstrap_ratio, nc_chroma_lag*, nc_window_energy_blocks and the
 *         chroma plan / tail and trim bounds inside the larger ones: two one-thread marker
 *         launches each, timeline diagnosis only); on = 0: off.
 * nc_profile_read(tag) waits for the recorded launches, returns their summed event
 * duration and count, and resets the tag's events.  nc_profile_read_span(tag) returns
 * the summed execution spans (first wave start .. last wave end on the device wall
 * clock: the duration rocprofv3 --kernel-trace reports, without the time a kernel
 * queues behind other streams' work) and resets the tag's spans.  Tags: "stft_mel",
 * "window_tg", "tuning_peaks", "decimate", "cqt_chroma", "trim_blocks", "tempo_beat",
 * "tg_slide", "spectral_frames", "spectral_bins".  Enabling (or disabling) discards
 * pending records.  nc_profile_read_busy (modes 1-3, 5) returns the union of every span
 * recorded since the last read, all tags together (device busy time), the extent from the
 * first start to the last end, and the number of spanned launches, and clears the spans:
 * 1 - busy / extent is the device's idle fraction over those launches. */
int nc_profile_enable(nc_ctx* ctx, int on);
int nc_profile_read(nc_ctx* ctx, const char* tag, double* total_ms, int* launches);
int nc_profile_read_span(nc_ctx* ctx, const char* tag, double* total_ms, int* launches);
int nc_profile_read_busy(nc_ctx* ctx, double* busy_ms, double* extent_ms, int* launches);
/* nc_profile_dump_spans (modes 1-3): every span recorded since the last read, in launch order:
 * the launch's tag index into `tags` (the tag names written '\n'-separated, NUL-terminated, at
 * most tags_cap bytes), its start and end in ms from the earliest start; at most cap spans,
 * *n = how many.  Clears the spans (as nc_profile_read_busy).  Measurement only: the untraced
 * timeline of which kernels run together (tools/concurrency.py). */
int nc_profile_dump_spans(nc_ctx* ctx, char* tags, int tags_cap, int* tag_index, double* start_ms, double* end_ms,
                          int cap, int* n);

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

/* K1b' window energies from a finished nc_trim_bounds workspace (ABI 5) — replaces
 * io._rms_db (io.py:38-40) for windows of the trimmed files: window w of file
 * win_file[w] (an index into that trim call's files, whose untrimmed offsets are
 * file_off) at sig + win_off[w], win_len samples; energy_out[w] = RMS dB (f64) from
 * the trim's f64 512-sample block sums plus the partial blocks at the window ends.
 * The per-window stage then runs with energy_out = NULL (no per-frame energy). */
int nc_window_energy_blocks(nc_ctx* ctx, const float* sig, const void* trim_ws, int n_files, const int64_t* file_off,
                            const int64_t* win_off, const int* win_file, int n_win, int win_len, double* energy_out,
                            void* stream);

/* ---------------------------------------------------------------------------
 * K1b+K2..K5  per-window stage — replaces io._rms_db (io.py:38-40) and, inside
 * tempo.estimate_tempo (tempo.py:27-77), librosa.onset.onset_strength
 * (tempo.py:44) and the tempogram mean behind beat_track/feature.tempo
 * (tempo.py:45-50, 61-68).
 * Window w = win_len samples at sig + win_off[w] (hop must be 512).
 * Outputs: onset_out[w*T + t] (T = 1 + win_len/512), tg_out[w*acw + k]
 * (acw = 344: mean over frames of the inf-normalised tempogram),
 * energy_out[w] (RMS dB, float64; nullable since ABI 5: then no energy is computed,
 * nc_window_energy_blocks gives it from the trim).  `active` (nullable) skips windows.
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


/* ---------------------------------------------------------------------------
 * K9..K11  CQT chroma — replaces pitch._mean_chroma (pitch.py:55-64) =
 * librosa.feature.chroma_cqt(y, sr=22050, bins_per_octave=36, hop_length=512)
 * .mean(axis=1) for each chunk c = sig[chunk_off[c] .. +chunk_len[c]):
 * tuning estimate (piptrack, 0.01-bin histogram) -> 7-octave CQT (252 bins,
 * octave decimation by the engine's half-band FIR in place of soxr_hq) ->
 * 12-bin chroma (n_chroma = 12: the reference's lag/3 quirk) ->
 * per-frame inf-norm -> mean.  out_chroma[c*12 + k] (f32), out_tuning[c]
 * (f32, bins), out_tuning_idx[c] (nullable; index on the 0.01 grid),
 * out_tuning_margin[c] (nullable; the tuning decision's margin: the argmax bin's
 * residual count minus the runner-up's, 0 on a tie broken by np.argmax's first-index
 * rule, 0 when no peak passes the threshold).
 * total_len = sum of chunk_len; max_chunk_len = max of chunk_len.
 * ------------------------------------------------------------------------- */
size_t nc_chroma_workspace_bytes(const nc_ctx* ctx, int n_chunks, int64_t total_len);
int nc_chroma_mean(nc_ctx* ctx, const float* sig, const int64_t* chunk_off, const int64_t* chunk_len,
                   int n_chunks, int64_t total_len, int64_t max_chunk_len, float* out_chroma,
                   float* out_tuning, int* out_tuning_idx, int* out_tuning_margin, void* ws, size_t ws_bytes,
                   void* stream);

/* ---------------------------------------------------------------------------
 * K9-K11 with shared tuning frames (optional fusion; same results as the pair
 * nc_window_stage + nc_chroma_mean).  The first tp_frames tuning frames (2048 / 512,
 * centred) of a 20 s chunk that starts where a 10 s window starts are that window's
 * own STFT frames: same samples, same zero padding on the left, none on the right
 * while t * 512 + 1024 <= win_len (tp_frames = 429 for 10 s windows).
 * nc_window_stage_tuning = nc_window_stage that also runs estimate_tuning's piptrack
 * (pitch.py:58 -> librosa.estimate_tuning) on those frames: win_chunk[w] = the chunk
 * window w starts (or -1), chunk_tf_base[c] = sum_{q<c} (1 + chunk_len[q] / 512) (the
 * chunk's slot base in the peak lists, in units of 192 slots), peak_pitch / peak_mag =
 * chunk_tf_base[n] * 192 floats each (peak_mag holds 2x piptrack's magnitude, exactly:
 * only its median and comparisons are consumed), chunk_npk[n] zeroed by the caller.  If
 * stft_done_event (a hipEvent_t) is given it is recorded once the peaks are written.
 * nc_chroma_mean_shared = nc_chroma_mean on the same peak lists: tuning frames
 * t < tf_skip[c] are not recomputed (tf_skip_total = sum of tf_skip, host value), the
 * counts are not zeroed, and the stream waits for wait_event before the tuning select.
 * ------------------------------------------------------------------------- */
int nc_window_stage_tuning(nc_ctx* ctx, const float* sig, const int64_t* win_off, const uint8_t* active,
                           int n_win, int win_len, int hop, float* onset_out, double* tg_out,
                           double* energy_out, const int* win_chunk, const int64_t* chunk_tf_base,
                           int tp_frames, float* peak_pitch, float* peak_mag, int* chunk_npk,
                           void* stft_done_event, void* ws, size_t ws_bytes, void* stream);
int nc_chroma_mean_shared(nc_ctx* ctx, const float* sig, const int64_t* chunk_off, const int64_t* chunk_len,
                          int n_chunks, int64_t total_len, int64_t max_chunk_len, float* out_chroma,
                          float* out_tuning, int* out_tuning_idx, int* out_tuning_margin, const int* tf_skip,
                          int64_t tf_skip_total,
                          float* peak_pitch, float* peak_mag, int* chunk_npk, void* wait_event, void* ws,
                          size_t ws_bytes, void* stream);
/* pitch._cyclic_xcorr_peak (pitch.py:67-85): lag_out[p] = wrapped argmax_k
 * dot(chroma[src_idx[p]], roll(chroma[nc_idx[p]], -k)), in [-5, 6]. */
int nc_chroma_lag(nc_ctx* ctx, const float* chroma, const int* src_idx, const int* nc_idx, int n_pairs,
                  int* lag_out, void* stream);
/* nc_chroma_lag plus margin_out[p] = (best - second best xcorr) / |best|: how far the
 * lag decision is from a tie (no reference equivalent; diagnostics). */
int nc_chroma_lag_margin(nc_ctx* ctx, const float* chroma, const int* src_idx, const int* nc_idx, int n_pairs,
                         int* lag_out, double* margin_out, void* stream);
/* pitch._cyclic_xcorr_peak (pitch.py:67-85) for vectors of any length n >= 1: pair p is
 * src[p*n .. p*n+n) against nc[p*n .. p*n+n); lag_out[p] = argmax_k dot(src, roll(nc, -k))
 * (first maximum, first NaN wins as np.argmax), minus n when it exceeds n / 2. */
int nc_xcorr_peak(nc_ctx* ctx, const float* src, const float* nc, int n, int n_pairs, int* lag_out, void* stream);

/* ---------------------------------------------------------------------------
 * device glue between the kernels (so a batch needs no host round trip)
 * nc_energy_gate   io.energy_gate (io.py:115-126) per group of windows
 *                  [w0[g], w1[g]): active[w] = energy_db[w] >= max + threshold_db
 * nc_collect_valid consensus._valid (consensus.py:236-240) of the per-window
 *                  tempo lists: in window order, values of windows that are
 *                  active, have nbeats >= min_beats (tempo.py:54-55) and a finite
 *                  positive bpm -> out_values[w0[g] + i], count out_n[g]
 * nc_pitch_hz      pitch.py:95,161-164: shift = lag/3.0, nc_hz = 440*2^(shift/12),
 *                  src_hz = 440
 * ------------------------------------------------------------------------- */
/* io._rms_db (io.py:38-40) alone, for windows sig[win_off[w] .. +win_len) */
int nc_window_energy(nc_ctx* ctx, const float* sig, const int64_t* win_off, int n_win, int win_len,
                     double* energy_out, void* stream);
int nc_energy_gate(nc_ctx* ctx, const double* energy_db, const int* w0, const int* w1, int n_groups,
                   double threshold_db, uint8_t* active_out, void* stream);
int nc_collect_valid(nc_ctx* ctx, const double* bpm, const int* nbeats, const uint8_t* active,
                     const int* w0, const int* w1, int n_groups, int min_beats, double* out_values,
                     int* out_n, void* stream);
int nc_pitch_hz(nc_ctx* ctx, const int* lags, int n, double* shift_out, double* nc_hz, double* src_hz,
                void* stream);

/* ---------------------------------------------------------------------------
 * K12  bootstrap ratio of medians — replaces consensus._bootstrap_ratio
 * (consensus.py:243-267), consensus.compute_ibi_ratio (consensus.py:270-312)
 * and the chunk-shift bootstrap of pitch.estimate_pitch_chroma
 * (pitch.py:143-150).  Job j draws A = values[a_off[j] .. +a_n[j]) first and
 * B = values[b_off[j] .. +b_n[j]) second (b_off/b_n NULL: single array) with
 * numpy Generator(PCG64) choice(replace=True) semantics, bit-exact:
 * seed[j*4 .. +4] = PCG64 {state_hi, state_lo, inc_hi, inc_lo} of
 * np.random.default_rng(seed).  boot[i] = median(A*)/median(B*) (median(A*));
 * point = median(A)/median(B); CI = numpy 'linear' percentiles given as
 * (virtual index, gamma) pairs for the low and high quantile.  Jobs with
 * a_n < min_n (or b_n < min_n) yield NaN (the reference's MIN_VALID gate).
 * Workspace: job j uses job_cap[j] (>= a_n + b_n) values at byte offset
 * job_ws_off[j]; size each with nc_bootstrap_job_bytes(cap, n_boot).
 * ------------------------------------------------------------------------- */
size_t nc_bootstrap_job_bytes(int cap, int n_boot);
int nc_bootstrap_ratio(nc_ctx* ctx, const double* values, const int64_t* a_off, const int* a_n,
                       const int64_t* b_off, const int* b_n, int n_jobs, int n_boot,
                       const uint64_t* seed, double idx_lo, double gamma_lo, double idx_hi,
                       double gamma_hi, int min_n, double* point_out, double* lo_out, double* hi_out,
                       double* boot_out, const int64_t* job_ws_off, const int* job_cap, void* ws,
                       size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * hop-64 IBI pass, part 1 — librosa.onset.onset_strength(y, sr, hop_length=hop)
 * over whole files (tempo.py:158): file f = sig[file_off[f] .. +file_len[f]),
 * onset_out at frame_base[f] (frame_base_out[n_files+1], written here:
 * prefix of 1 + file_len/hop).  total_frames = sum(1 + file_len/hop).
 * ------------------------------------------------------------------------- */
size_t nc_ibi_onset_workspace_bytes(const nc_ctx* ctx, int n_files, int64_t total_frames);
int nc_ibi_onset(nc_ctx* ctx, const float* sig, const int64_t* file_off, const int64_t* file_len,
                 int n_files, int64_t total_frames, int hop, float* onset_out,
                 int64_t* frame_base_out, void* ws, size_t ws_bytes, void* stream);
/* part 2 — the tempogram mean (win_length = ac_size*sr/hop, 2756 at hop 64)
 * that beat_track argmaxes (tempo.py:159), streamed instead of materialised:
 * tg_out[f*acw + k].  total_frames = frame_base[n_files]; max_frames = the
 * largest per-file frame count (sizes the tile grid). */
size_t nc_ibi_tempogram_workspace_bytes(const nc_ctx* ctx, int n_files, int64_t total_frames, int max_frames,
                                        int hop);
int nc_ibi_tempogram(nc_ctx* ctx, const float* onset, const int64_t* frame_base, int n_files,
                     int64_t total_frames, int max_frames, int hop, double* tg_out, void* ws, size_t ws_bytes,
                     void* stream);
/* The same pass split over ranks (window-sharded runs); one rank's
 * share of file f is frames [t0[f], t1[f]) and tempogram tiles [b0[f], b1[f]) (2048 frames
 * each); t0 / t1 / b0 / b1 are device int64 arrays.
 * nc_ibi_mel_range:   the mel dB rows the onsets of [t0, t1) need (STFT frames
 *                     [t0 - pad, t1 - pad + 1) within the file, pad = 1 + 1024 / hop) into ws,
 *                     and max_out[f] = their largest dB value (-inf for none): this rank's
 *                     share of power_to_db's top_db reference (C2: all-reduce MAX).
 *                     total_rows = the host's count of those rows over all files.
 * nc_ibi_onset_range: onset_out[obase[f] + t - t0[f]] for t in [t0[f], t1[f]) (obase =
 *                     prefix of t1 - t0; total_out = its sum) against the file's global
 *                     maximum gmax[f]; ws and total_rows as in the nc_ibi_mel_range call.
 *                     (C4: the segments are gathered into each file's full onset.)
 * nc_ibi_tempogram_tiles:  partial rows slab[(f * n_tblk + b) * N + k] of tiles
 *                     b in [b0[f], b1[f]) from the FULL onset (n_tblk = ceil(max_frames / 2048),
 *                     N = tempogram window); ws sized by nc_ibi_tempogram_workspace_bytes.
 * nc_ibi_tempogram_reduce: tg_out[f * N + k] = (sum over b of slab rows, in order) / T_f
 *                     once every tile's row is in slab (C3: the rows are gathered) -- the
 *                     same bits as nc_ibi_tempogram. */
size_t nc_ibi_range_workspace_bytes(const nc_ctx* ctx, int n_files, int64_t total_rows);
int nc_ibi_mel_range(nc_ctx* ctx, const float* sig, const int64_t* file_off, const int64_t* file_len,
                     int n_files, const int64_t* t0, const int64_t* t1, int hop, int64_t total_rows,
                     float* max_out, void* ws, size_t ws_bytes, void* stream);
int nc_ibi_onset_range(nc_ctx* ctx, int n_files, const int64_t* t0, int hop, int64_t total_out,
                       const float* gmax, float* onset_out, void* ws, int64_t total_rows, void* stream);
int nc_ibi_tempogram_tiles(nc_ctx* ctx, const float* onset, const int64_t* frame_base, int n_files,
                           int64_t total_frames, int max_frames, int hop, const int64_t* b0, const int64_t* b1,
                           double* slab, void* ws, size_t ws_bytes, void* stream);
int nc_ibi_tempogram_reduce(nc_ctx* ctx, const double* slab, const int64_t* frame_base, int n_files,
                            int max_frames, int hop, double* tg_out, void* stream);

/* ---------------------------------------------------------------------------
 * K13  windowed waveform cross-correlation — the search loop of
 * xcorr.estimate_speed_xcorr (xcorr.py:109-160).  The caller plans the
 * reference's integer geometry: n_items dot products of `win` samples between
 * sig[item_a[i]..] and sig[item_b[i]..]; job j owns windows [w0[j], w1[j]);
 * window w has its self item win_self[w] (a.a), candidate items
 * [cand0[w], cand1[w]) whose b positions are pb[item], its a position pa[w]
 * and default exp_pb[w].  Outputs ratio_out[j] (np.polyfit slope) and
 * quality_out[j] (median normalised correlation); (1, 0) with < 3 matches.
 * scratch: dot/sqb = 2 * n_items doubles (caller-owned device memory).
 * ------------------------------------------------------------------------- */
int nc_xcorr_search(nc_ctx* ctx, const float* sig, const int64_t* item_a, const int64_t* item_b,
                    int n_items, int win, double* dot, double* sqb, const int* w0, const int* w1,
                    const int* win_self, const int* cand0, const int* cand1, const int64_t* pa,
                    const int64_t* pb, const int64_t* exp_pb, int n_jobs, double* ratio_out,
                    double* quality_out, void* stream);

/* ---------------------------------------------------------------------------
 * intro offset of pipeline.run(auto_align=True) — xcorr.find_content_offset
 * (xcorr.py:165-259; called at pipeline.py:111-125) for n_pairs (src, nc)
 * pairs of 22050 Hz signals (sig[src_off[p] ..], src_len[p] samples; likewise
 * nc): 2:1 resample to 11025 Hz, RMS envelopes (frame 2048, hop 512), for each
 * of n_speeds candidate speeds (device f64, the reference's np.linspace(1.03,
 * 1.5, 30)) the nc envelope stretched to int(len / speed) frames by np.interp
 * and correlated with the first max_offset_frames + 1 lags of the src envelope
 * (int(120 / (512 / 11025)) = 2583 in the reference); the cosine score of each
 * speed's first argmax decides, first best wins.  Outputs per pair: peak lag
 * (offset_sec = peak * 512 / 11025), speed index (-1: no speed searchable,
 * the reference then returns (0.0, (lo + hi) / 2)) and the score.
 * total_len = sum of all 2 n_pairs lengths, max_len = the longest (grid and
 * workspace sizing); size ws with nc_align_workspace_bytes.
 * ------------------------------------------------------------------------- */
size_t nc_align_workspace_bytes(const nc_ctx* ctx, int n_pairs, int n_speeds, int64_t total_len,
                                int64_t max_len, int max_offset_frames);
int nc_align_offsets(nc_ctx* ctx, const float* sig, const int64_t* src_off, const int64_t* src_len,
                     const int64_t* nc_off, const int64_t* nc_len, int n_pairs, const double* speeds,
                     int n_speeds, int max_offset_frames, int64_t total_len, int64_t max_len,
                     int* peak_out, int* speed_idx_out, double* score_out, void* ws, size_t ws_bytes,
                     void* stream);

/* ---------------------------------------------------------------------------
 * S1  spectral statistics — replaces, inside spectral.analyze (spectral.py:38-103),
 *     librosa.feature.spectral_centroid (:54), spectral_rolloff(roll_percent) (:55-57),
 *     feature.rms (:59, :76), the |stft| band means (:63-74) and
 *     amplitude_to_db(|stft|, ref=np.max) averaged over time (:87-88).
 * File f = file_len[f] samples at sig + file_off[f], at its own sample rate (the
 * reference loads with sr=None, :52).  STFT 2048 / hop 512, periodic Hann, centred,
 * zero pad: T_f = 1 + file_len[f] / 512 frames, frame_base[f] = sum_{q<f} T_q
 * (device, n_files + 1 entries; total_frames = frame_base[n_files], max_frames =
 * max T_f).  bin_hz[f] = np.fft.rfftfreq(2048, 1/sr)[1] (f64, device);
 * band_bins[f*10 + 2b], [f*10 + 2b + 1] = the [lo, hi) bins of band b's mask
 * (freqs >= lo_hz) & (freqs < hi_hz) for the bands 20-80, 80-250, 250-2000,
 * 2000-6000, 6000-20000 Hz.
 * Outputs: rms_out[frame_base[f] + t] = frame RMS (f32); stats_out[f*12 + i] =
 * {sum_t centroid_t, sum_t rolloff_t (Hz), 5 x sum_t sum_{k in band} |S|, max |S|,
 * mean(rms), var(rms), np.percentile(rms, 75), mean(diff(rms[rms > p75]))};
 * bin_db_out[f*1025 + k] = sum_t max(dB(|S|^2) - dB(ref^2), -80).  The host
 * divides by T_f (and by the band bin counts) and thresholds the bin means.
 * Size ws with nc_spectral_workspace_bytes.
 * ------------------------------------------------------------------------- */
size_t nc_spectral_workspace_bytes(int64_t total_frames, int n_files, int64_t max_frames);
int nc_spectral_stats(nc_ctx* ctx, const float* sig, const int64_t* file_off, const int64_t* file_len,
                      const int64_t* frame_base, const double* bin_hz, const int* band_bins, int n_files,
                      int64_t total_frames, int64_t max_frames, float roll_percent, float* rms_out,
                      double* stats_out, double* bin_db_out, void* ws, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------
 * R1  load-time resampler — replaces the resample inside io.load_audio
 *     (io.py:44-55: librosa.load(path, sr=22050) -> soxr_hq) for files that are
 *     not at 22 050 Hz.  libsoxr is absent and cannot be bit-matched; the engine's
 *     stand-in is scipy.signal.resample_poly(x, up, down) (Kaiser(5.0) FIR,
 *     constant zero padding), reproduced bit for bit in f64.  For each file f:
 *     y[out_off[f] + m] = upfirdn(h, x[in_off[f] ..], up, down)[m + pre_remove]
 *     (float), m < out_len[f] = ceil(in_len[f] up / down); max_out = max out_len.
 *     h (device f64, h_len = a multiple of up) is resample_poly's filter:
 *     firwin(20 max(up,down) + 1, 1/max(up,down), ('kaiser', 5)) * up, with its
 *     leading / trailing zero padding; pre_remove = resample_poly's n_pre_remove.
 *     All files of one call share (up, down, h).
 * ------------------------------------------------------------------------- */
int nc_resample_poly(nc_ctx* ctx, const float* x, const int64_t* in_off, const int64_t* in_len, int n_files,
                     float* y, const int64_t* out_off, const int64_t* out_len, int64_t max_out,
                     const double* h, int h_len, int up, int down, int64_t pre_remove, void* stream);

/* -------------------------------------------------------------------------
 * R1b 16-bit PCM upload — replaces the int16 -> float32 scaling inside
 *     io.load_audio (io.py:44-55: librosa.load -> soundfile, sample k -> k / 32768)
 *     for mono 16-bit WAV files: the host uploads the stored 2-byte samples and
 *     y[i] = x[i] / 32768 (exact in f32) is computed in HBM.  x and y 16-byte
 *     aligned, n samples.  (ABI 5)
 * ------------------------------------------------------------------------- */
int nc_pcm16_to_f32(nc_ctx* ctx, const int16_t* x, int64_t n, float* y, void* stream);

/* -------------------------------------------------------------------------
 * MELODIA front end (opt-in; replaces the frame-level part of essentia's
 * PredominantPitchMelodia that pitch.estimate_pitch_melodia calls,
 * pitch.py:210-215: frameSize 2048, hopSize 128).  PARITY UNPINNED: essentia is
 * not installed here; the CPU restatement is oracle/melodia_ref.py.
 *
 * nc_melodia_salience: for every frame t < n_frames[f] of every file f (frame g
 * = frame_base[f] + t; n_frames = ceil((len + 1024) / hop), frames centred at
 * t hop): the 2048-sample frame times win (2048 floats, device: essentia's
 * normalised symmetric Hann), zero-padded to 8192 -> |X| -> the 100 largest
 * spectral peaks (parabolic interpolation) -> the 600-bin, 10-cent pitch
 * salience from 55 Hz (20 harmonics, weight 0.8^h, cos^2 over +-1 semitone,
 * peaks within 40 dB of the frame's largest) -> its local maxima in bins
 * [sal_min_bin, 599], the NC_MELODIA_SALPK largest:
 *   pk_count[g], pk_bin[g * NC_MELODIA_SALPK + i] (int), pk_sal[...] (float),
 *   i < pk_count[g], ordered by salience (descending), ties by bin.
 * frame_base: device int64 [n_files + 1].  No workspace.
 * ------------------------------------------------------------------------- */
#define NC_MELODIA_SALPK 128
int nc_melodia_salience(nc_ctx* ctx, const float* sig, const int64_t* file_off, const int64_t* file_len,
                        const int64_t* frame_base, int n_files, int64_t total_frames, int hop, float sample_rate,
                        const float* win, int sal_min_bin, int* pk_count, int* pk_bin, float* pk_sal,
                        void* stream);

#ifdef __cplusplus
}
#endif
#endif /* NCGPU_H */
