// nc_capi.cpp — extern "C" entry points of libncgpu.so (declared in include/ncgpu.h).
#include <cstdlib>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>

#include "../../include/ncgpu.h"
#include "nc_engine.h"

namespace nc {

thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }

// kernels (defined in the .hip translation units)
int launch_melodia_salience(Context& ctx, const float* sig, const int64_t* file_off, const int64_t* file_len,
                            const int64_t* frame_base, int n_files, int64_t total_frames, int hop, float sr,
                            const float* win, int sal_min_bin, int* pk_count, int* pk_bin, float* pk_sal,
                            hipStream_t st);
struct BeatArgs;
size_t window_stage_ws_bytes(const Context& ctx, int n_win, int T);
int launch_window_stage(Context& ctx, const float* sig, const int64_t* win_off, const uint8_t* active,
                        int n_win, int win_len, int hop, float* onset_out, double* tg_out,
                        double* energy_out, const int* win_chunk, const int64_t* chunk_tf_base, int tp_frames,
                        float* peak_pitch, float* peak_mag, int* chunk_npk, void* stft_done,
                        void* ws, size_t ws_bytes, hipStream_t st);
int launch_tempo_beats_c(Context& ctx, const float* onset, const int64_t* off, const int* len, int n_seq,
                         int max_len, const double* tg, int acw, const double* start_bpm,
                         const int* prior_idx, const uint8_t* active, int hop, int trim, double* bpm_out,
                         int* lag_out, int* nbeats_out, double* margin_out, int* beats_out,
                         int64_t total_frames, void* ws, size_t ws_bytes, hipStream_t st);
int launch_nc_prior(const double* bpm, const int* nbeats, const uint8_t* active, const int* src_w0,
                    const int* src_w1, const int64_t* src_len, const int64_t* nc_len, int n_pairs,
                    double* prior_out, hipStream_t st, int sr);
int launch_ibi_from_beats(const int* beats, const int64_t* off, const int* nbeats, int n_seq, int hop,
                          int min_ibis, double* ibi_out, int* n_ibi, hipStream_t st, int sr);
size_t trim_ws_bytes(const int64_t* host_file_len, int n_files);
int launch_trim(Context& ctx, const float* sig, const int64_t* file_off, const int64_t* file_len, int n_files,
                int64_t max_frames, float top_db, int64_t* out_start, int64_t* out_end, void* ws,
                size_t ws_bytes, hipStream_t st);

size_t chroma_ws_bytes(int n, int64_t total_len);
int launch_chroma_mean(Context& ctx, const float* sig, const int64_t* chunk_off, const int64_t* chunk_len, int n,
                       int64_t total_len, int64_t max_chunk_len, float* out_chroma, float* out_tuning,
                       int* out_tuning_idx, int* out_tuning_margin, const int* tf_skip, int64_t tf_skip_total,
                       float* ext_pitch,
                       float* ext_mag, int* ext_npk, void* wait_event, void* ws, size_t ws_bytes, hipStream_t st);
int launch_chroma_lag(const float* chroma, const int* src_idx, const int* nc_idx, int n_pairs, int* lag_out,
                      double* margin_out, hipStream_t st);
int launch_xcorr_peak(const float* a, const float* b, int n, int n_pairs, int* lag_out, hipStream_t st);

size_t bootstrap_job_bytes(int cap, int n_boot);
int launch_bootstrap(const BootArgs& a, int n_jobs, hipStream_t st);

size_t ibi_onset_ws_bytes(int n_files, int64_t total_frames);
int launch_ibi_onset(Context& ctx, const float* sig, const int64_t* file_off, const int64_t* file_len, int n_files,
                     int64_t total_frames, int hop, float* onset_out, int64_t* frame_base_out, void* ws,
                     size_t ws_bytes, hipStream_t st);
size_t ibi_tg_ws_bytes(const Context& ctx, int n_files, int64_t total_frames, int max_frames, int hop);
int launch_ibi_tempogram(Context& ctx, const float* onset, const int64_t* frame_base, int n_files,
                         int64_t total_frames, int max_frames, int hop,
                         double* tg_out, void* ws, size_t ws_bytes, hipStream_t st);

size_t ibi_range_ws_bytes(int n_files, int64_t total_rows);
int launch_ibi_mel_range(Context& ctx, const float* sig, const int64_t* file_off, const int64_t* file_len,
                         int n_files, const int64_t* t0, const int64_t* t1, int hop, int64_t total_rows,
                         float* max_out, void* ws, size_t ws_bytes, hipStream_t st);
int launch_ibi_onset_range(int n_files, const int64_t* t0, int hop, int64_t total_out, const float* gmax,
                           float* onset_out, void* ws, int64_t total_rows, hipStream_t st);
int launch_ibi_tempogram_tiles(Context& ctx, const float* onset, const int64_t* frame_base, int n_files,
                               int64_t total_frames, int max_frames, int hop, const int64_t* b0, const int64_t* b1,
                               double* slab_out, double* tg_out, void* ws, size_t ws_bytes, hipStream_t st);
int launch_ibi_tempogram_reduce(Context& ctx, const double* slab, const int64_t* frame_base, int n_files,
                                int max_frames, int hop, double* tg_out, hipStream_t st);

size_t align_ws_bytes(int n_pairs, int n_speeds, int64_t total_len, int64_t max_len, int max_off_frames);
int launch_align_offsets(Context& ctx, const float* sig, const int64_t* src_off, const int64_t* src_len,
                         const int64_t* nc_off, const int64_t* nc_len, int n_pairs, const double* speeds,
                         int n_speeds, int max_off_frames, int64_t total_len, int64_t max_len, int* out_peak,
                         int* out_speed, double* out_score, void* ws, size_t ws_bytes, hipStream_t st);
int launch_xcorr(const float* sig, const int64_t* ia, const int64_t* ib, int n_items, int win, double* dot,
                 double* sqb, const int* w0, const int* w1, const int* sw, const int* c0, const int* c1,
                 const int64_t* pa, const int64_t* pbv, const int64_t* exp_pb, int n_jobs, double* ratio_out,
                 double* quality_out, hipStream_t st);

size_t spectral_ws_bytes(int64_t total_frames, int n_files, int64_t max_frames);
int launch_spectral(Context& ctx, const float* sig, const int64_t* file_off, const int64_t* file_len,
                    const int64_t* frame_base, const double* bin_hz, const int* band_bins, int n_files,
                    int64_t total_frames, int64_t max_frames, float roll_percent, float* rms_out,
                    double* stats_out, double* bin_db_out, void* ws, size_t ws_bytes, hipStream_t st);

int launch_pcm16_to_f32(const int16_t* x, int64_t n, float* y, hipStream_t st);
int launch_window_energy_blocks(const float* sig, const void* trim_ws, int n_files, const int64_t* file_off,
                                const int64_t* win_off, const int* win_file, int n_win, int win_len, double* out,
                                hipStream_t st);
int launch_resample_poly(const float* x, const int64_t* in_off, const int64_t* in_len, int n_files,
                         float* y, const int64_t* out_off, const int64_t* out_len, int64_t max_out,
                         const double* h, int h_len, int up, int down, int64_t pre_remove, hipStream_t st);

int launch_energy_gate(const double* energy, const int* w0, const int* w1, int n_groups, double gate_db,
                       uint8_t* active, hipStream_t st);
int launch_collect_valid(const double* bpm, const int* nbeats, const uint8_t* active, const int* w0, const int* w1,
                         int n_groups, int min_beats, double* out_values, int* out_n, hipStream_t st);
int launch_pitch_hz(const int* lags, int n, double* shift_out, double* nc_hz, double* src_hz, hipStream_t st);
int launch_window_energy(const float* sig, const int64_t* off, int n, int win_len, double* out, hipStream_t st);

}  // namespace nc

struct nc_ctx {
  nc::Context c;
};

#define CHECK_CTX(ctx)                         \
  do {                                         \
    if (!(ctx)) {                              \
      nc::set_error("null context");           \
      return -1;                               \
    }                                          \
  } while (0)

#define SET_DEVICE(ctx)                                                              \
  do {                                                                               \
    hipError_t _e = hipSetDevice((ctx)->c.device);                                   \
    if (_e != hipSuccess) {                                                          \
      nc::set_error(std::string("hipSetDevice: ") + hipGetErrorString(_e));          \
      return -1;                                                                     \
    }                                                                                \
  } while (0)

extern "C" {

int nc_abi_version(void) { return NCGPU_ABI_VERSION; }
const char* nc_last_error(void) { return nc::g_err.c_str(); }

int nc_create(int device, nc_ctx** out) { return nc_create_rate(device, nc::kSR, out); }

int nc_create_rate(int device, int sample_rate, nc_ctx** out) {
  if (!out) {
    nc::set_error("nc_create: null out");
    return -1;
  }
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
    nc::set_error("nc_create: no HIP device visible");
    return -1;
  }
  if (device < 0 || device >= ndev) {
    nc::set_error("nc_create: bad device index");
    return -1;
  }
  NC_HIP(hipSetDevice(device));
  if (sample_rate < 8000 || sample_rate > 48000) {
    nc::set_error("nc_create_rate: sample rate outside 8000..48000 Hz");
    return -2;
  }
  nc_ctx* c = new nc_ctx();
  c->c.device = device;
  c->c.sr = sample_rate;
  int cu = 0;
  if (hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cu > 0)
    c->c.num_cu = cu;
  if (const char* v = std::getenv("NC_STFT_CUS")) c->c.stft_cus = std::max(0, std::atoi(v));
  if (const char* v = std::getenv("NC_CHROMA_CUS")) c->c.chroma_cus = std::max(0, std::atoi(v));
  nc::build_tables(c->c);
  if (!c->c.t.tw || !c->c.t.cqt_w || !c->c.t.halfband) {
    nc::free_tables(c->c);
    delete c;
    nc::set_error("nc_create: table allocation failed");
    return -1;
  }
  *out = c;
  return 0;
}

int nc_destroy(nc_ctx* ctx) {
  CHECK_CTX(ctx);
  (void)hipSetDevice(ctx->c.device);
  nc::free_timers(ctx->c);
  nc::free_tables(ctx->c);
  delete ctx;
  return 0;
}

int nc_num_cu(const nc_ctx* ctx) { return ctx ? ctx->c.num_cu : -1; }

int nc_profile_enable(nc_ctx* ctx, int on) {
  CHECK_CTX(ctx);
  SET_DEVICE(ctx);
  if (on < 0 || on > 5) {
    nc::set_error("nc_profile_enable: mode must be 0 (off), 1 (events + spans), 2 (spans only), 3 "
                  "(events around the roofline kernels + spans), 4 (events around the roofline kernels) or 5 "
                  "(spans + marker spans around the small entry points)");
    return -1;
  }
  nc::profile_enable(ctx->c, on);
  return 0;
}

int nc_profile_read(nc_ctx* ctx, const char* tag, double* total_ms, int* launches) {
  CHECK_CTX(ctx);
  if (!tag || !total_ms || !launches) {
    nc::set_error("nc_profile_read: null argument");
    return -1;
  }
  SET_DEVICE(ctx);
  return nc::profile_read(ctx->c, tag, total_ms, launches);
}

int nc_profile_read_span(nc_ctx* ctx, const char* tag, double* total_ms, int* launches) {
  CHECK_CTX(ctx);
  if (!tag || !total_ms || !launches) {
    nc::set_error("nc_profile_read_span: null argument");
    return -1;
  }
  SET_DEVICE(ctx);
  return nc::profile_read_span(ctx->c, tag, total_ms, launches);
}

int nc_profile_read_busy(nc_ctx* ctx, double* busy_ms, double* extent_ms, int* launches) {
  CHECK_CTX(ctx);
  if (!busy_ms || !extent_ms || !launches) {
    nc::set_error("nc_profile_read_busy: null argument");
    return -1;
  }
  SET_DEVICE(ctx);
  return nc::profile_read_busy(ctx->c, busy_ms, extent_ms, launches);
}

int nc_profile_dump_spans(nc_ctx* ctx, char* tags, int tags_cap, int* tag_index, double* start_ms, double* end_ms,
                          int cap, int* n) {
  CHECK_CTX(ctx);
  if (!tags || tags_cap <= 0 || !tag_index || !start_ms || !end_ms || !n || cap < 0) {
    nc::set_error("nc_profile_dump_spans: null argument");
    return -1;
  }
  SET_DEVICE(ctx);
  return nc::profile_dump_spans(ctx->c, tags, tags_cap, tag_index, start_ms, end_ms, cap, n);
}

size_t nc_trim_workspace_bytes(const int64_t* host_file_len, int n_files) {
  return nc::trim_ws_bytes(host_file_len, n_files);
}

int nc_trim_bounds(nc_ctx* ctx, const float* sig, const int64_t* file_off, const int64_t* file_len, int n_files,
                   int64_t max_frames, float top_db, int64_t* out_start, int64_t* out_end, void* ws,
                   size_t ws_bytes, void* stream) {
  CHECK_CTX(ctx);
  SET_DEVICE(ctx);
  return nc::launch_trim(ctx->c, sig, file_off, file_len, n_files, max_frames, top_db, out_start, out_end, ws,
                         ws_bytes, (hipStream_t)stream);
}

size_t nc_window_stage_workspace_bytes(const nc_ctx* ctx, int n_win, int win_len, int hop) {
  if (!ctx || hop <= 0) return 0;
  return nc::window_stage_ws_bytes(ctx->c, n_win, 1 + win_len / hop);
}

int nc_window_stage(nc_ctx* ctx, const float* sig, const int64_t* win_off, const uint8_t* active, int n_win,
                    int win_len, int hop, float* onset_out, double* tg_out, double* energy_out, void* ws,
                    size_t ws_bytes, void* stream) {
  CHECK_CTX(ctx);
  SET_DEVICE(ctx);
  return nc::launch_window_stage(ctx->c, sig, win_off, active, n_win, win_len, hop, onset_out, tg_out,
                                 energy_out, nullptr, nullptr, 0, nullptr, nullptr, nullptr, nullptr, ws, ws_bytes,
                                 (hipStream_t)stream);
}

int nc_window_stage_tuning(nc_ctx* ctx, const float* sig, const int64_t* win_off, const uint8_t* active, int n_win,
                           int win_len, int hop, float* onset_out, double* tg_out, double* energy_out,
                           const int* win_chunk, const int64_t* chunk_tf_base, int tp_frames, float* peak_pitch,
                           float* peak_mag, int* chunk_npk, void* stft_done_event, void* ws, size_t ws_bytes,
                           void* stream) {
  CHECK_CTX(ctx);
  SET_DEVICE(ctx);
  return nc::launch_window_stage(ctx->c, sig, win_off, active, n_win, win_len, hop, onset_out, tg_out,
                                 energy_out, win_chunk, chunk_tf_base, tp_frames, peak_pitch, peak_mag, chunk_npk,
                                 stft_done_event, ws, ws_bytes, (hipStream_t)stream);
}

size_t nc_tempo_beats_workspace_bytes(int64_t total_frames) {
  return (size_t)total_frames * (8 + 8 + 4 + 1) + 256;
}

int nc_tempo_beats(nc_ctx* ctx, const float* onset, const int64_t* off, const int* len, int n_seq, int max_len,
                   const double* tg, int acw, const double* start_bpm, const int* prior_idx,
                   const uint8_t* active, int hop, int trim, double* bpm_out, int* lag_out, int* nbeats_out,
                   double* margin_out, int* beats_out, int64_t total_frames, void* ws, size_t ws_bytes,
                   void* stream) {
  CHECK_CTX(ctx);
  SET_DEVICE(ctx);
  return nc::launch_tempo_beats_c(ctx->c, onset, off, len, n_seq, max_len, tg, acw, start_bpm, prior_idx, active,
                                  hop, trim, bpm_out, lag_out, nbeats_out, margin_out, beats_out, total_frames, ws,
                                  ws_bytes, (hipStream_t)stream);
}

int nc_tempo_prior(nc_ctx* ctx, const double* bpm, const int* nbeats, const uint8_t* active, const int* src_w0,
                   const int* src_w1, const int64_t* src_len, const int64_t* nc_len, int n_pairs,
                   double* prior_out, void* stream) {
  CHECK_CTX(ctx);
  SET_DEVICE(ctx);
  nc::MarkSpan ms_(ctx->c, "tempo_prior", (hipStream_t)stream);
  return nc::launch_nc_prior(bpm, nbeats, active, src_w0, src_w1, src_len, nc_len, n_pairs, prior_out,
                             (hipStream_t)stream, ctx->c.sr);
}

int nc_ibi_from_beats(nc_ctx* ctx, const int* beats, const int64_t* off, const int* nbeats, int n_seq, int hop,
                      int min_ibis, double* ibi_out, int* n_ibi, void* stream) {
  CHECK_CTX(ctx);
  SET_DEVICE(ctx);
  return nc::launch_ibi_from_beats(beats, off, nbeats, n_seq, hop, min_ibis, ibi_out, n_ibi,
                                   (hipStream_t)stream, ctx->c.sr);
}

size_t nc_chroma_workspace_bytes(const nc_ctx* ctx, int n_chunks, int64_t total_len) {
  (void)ctx;
  return nc::chroma_ws_bytes(n_chunks, total_len);
}

int nc_chroma_mean(nc_ctx* ctx, const float* sig, const int64_t* chunk_off, const int64_t* chunk_len, int n_chunks,
                   int64_t total_len, int64_t max_chunk_len, float* out_chroma, float* out_tuning,
                   int* out_tuning_idx, int* out_tuning_margin, void* ws, size_t ws_bytes, void* stream) {
  CHECK_CTX(ctx);
  SET_DEVICE(ctx);
  if (ctx->c.sr != nc::kSR) {
    nc::set_error("chroma: the CQT and tuning tables are built for 22050 Hz (nc_create)");
    return -2;
  }
  return nc::launch_chroma_mean(ctx->c, sig, chunk_off, chunk_len, n_chunks, total_len, max_chunk_len, out_chroma,
                                out_tuning, out_tuning_idx, out_tuning_margin, nullptr, 0, nullptr, nullptr, nullptr, nullptr, ws,
                                ws_bytes, (hipStream_t)stream);
}

int nc_chroma_mean_shared(nc_ctx* ctx, const float* sig, const int64_t* chunk_off, const int64_t* chunk_len,
                          int n_chunks, int64_t total_len, int64_t max_chunk_len, float* out_chroma,
                          float* out_tuning, int* out_tuning_idx, int* out_tuning_margin, const int* tf_skip,
                          int64_t tf_skip_total, float* peak_pitch, float* peak_mag, int* chunk_npk,
                          void* wait_event, void* ws, size_t ws_bytes, void* stream) {
  CHECK_CTX(ctx);
  SET_DEVICE(ctx);
  if (ctx->c.sr != nc::kSR) {
    nc::set_error("chroma: the CQT and tuning tables are built for 22050 Hz (nc_create)");
    return -2;
  }
  return nc::launch_chroma_mean(ctx->c, sig, chunk_off, chunk_len, n_chunks, total_len, max_chunk_len, out_chroma,
                                out_tuning, out_tuning_idx, out_tuning_margin, tf_skip, tf_skip_total, peak_pitch, peak_mag, chunk_npk,
                                wait_event, ws, ws_bytes, (hipStream_t)stream);
}

int nc_chroma_lag(nc_ctx* ctx, const float* chroma, const int* src_idx, const int* nc_idx, int n_pairs, int* lag_out,
                  void* stream) {
  CHECK_CTX(ctx);
  SET_DEVICE(ctx);
  nc::MarkSpan ms_(ctx->c, "chroma_lag", (hipStream_t)stream);
  return nc::launch_chroma_lag(chroma, src_idx, nc_idx, n_pairs, lag_out, nullptr, (hipStream_t)stream);
}

int nc_chroma_lag_margin(nc_ctx* ctx, const float* chroma, const int* src_idx, const int* nc_idx, int n_pairs,
                         int* lag_out, double* margin_out, void* stream) {
  CHECK_CTX(ctx);
  SET_DEVICE(ctx);
  nc::MarkSpan ms_(ctx->c, "chroma_lag", (hipStream_t)stream);
  return nc::launch_chroma_lag(chroma, src_idx, nc_idx, n_pairs, lag_out, margin_out, (hipStream_t)stream);
}

int nc_window_energy(nc_ctx* ctx, const float* sig, const int64_t* win_off, int n_win, int win_len,
                     double* energy_out, void* stream) {
  CHECK_CTX(ctx);
  SET_DEVICE(ctx);
  return nc::launch_window_energy(sig, win_off, n_win, win_len, energy_out, (hipStream_t)stream);
}

int nc_energy_gate(nc_ctx* ctx, const double* energy_db, const int* w0, const int* w1, int n_groups,
                   double threshold_db, uint8_t* active_out, void* stream) {
  CHECK_CTX(ctx);
  SET_DEVICE(ctx);
  nc::MarkSpan ms_(ctx->c, "energy_gate", (hipStream_t)stream);
  return nc::launch_energy_gate(energy_db, w0, w1, n_groups, threshold_db, active_out, (hipStream_t)stream);
}

int nc_collect_valid(nc_ctx* ctx, const double* bpm, const int* nbeats, const uint8_t* active, const int* w0,
                     const int* w1, int n_groups, int min_beats, double* out_values, int* out_n, void* stream) {
  CHECK_CTX(ctx);
  SET_DEVICE(ctx);
  nc::MarkSpan ms_(ctx->c, "collect_valid", (hipStream_t)stream);
  return nc::launch_collect_valid(bpm, nbeats, active, w0, w1, n_groups, min_beats, out_values, out_n,
                                  (hipStream_t)stream);
}

int nc_pitch_hz(nc_ctx* ctx, const int* lags, int n, double* shift_out, double* nc_hz, double* src_hz,
                void* stream) {
  CHECK_CTX(ctx);
  SET_DEVICE(ctx);
  nc::MarkSpan ms_(ctx->c, "pitch_hz", (hipStream_t)stream);
  return nc::launch_pitch_hz(lags, n, shift_out, nc_hz, src_hz, (hipStream_t)stream);
}

int nc_xcorr_peak(nc_ctx* ctx, const float* src, const float* nc, int n, int n_pairs, int* lag_out, void* stream) {
  CHECK_CTX(ctx);
  SET_DEVICE(ctx);
  return nc::launch_xcorr_peak(src, nc, n, n_pairs, lag_out, (hipStream_t)stream);
}

size_t nc_bootstrap_job_bytes(int cap, int n_boot) { return nc::bootstrap_job_bytes(cap, n_boot); }

int nc_bootstrap_ratio(nc_ctx* ctx, const double* values, const int64_t* a_off, const int* a_n, const int64_t* b_off,
                       const int* b_n, int n_jobs, int n_boot, const uint64_t* seed, double idx_lo, double gamma_lo,
                       double idx_hi, double gamma_hi, int min_n, double* point_out, double* lo_out, double* hi_out,
                       double* boot_out, const int64_t* job_ws_off, const int* job_cap, void* ws, size_t ws_bytes,
                       void* stream) {
  CHECK_CTX(ctx);
  SET_DEVICE(ctx);
  (void)ws_bytes;
  nc::BootArgs a;
  a.values = values;
  a.a_off = a_off;
  a.a_n = a_n;
  a.b_off = b_off;
  a.b_n = b_n;
  a.n_boot = n_boot;
  a.seed = seed;
  a.idx_lo = idx_lo;
  a.g_lo = gamma_lo;
  a.idx_hi = idx_hi;
  a.g_hi = gamma_hi;
  a.point_out = point_out;
  a.lo_out = lo_out;
  a.hi_out = hi_out;
  a.boot_out = boot_out;
  a.ws_off = job_ws_off;
  a.cap = job_cap;
  a.ws = static_cast<char*>(ws);
  a.min_n = min_n;
  nc::MarkSpan ms_(ctx->c, "bootstrap", (hipStream_t)stream);
  return nc::launch_bootstrap(a, n_jobs, (hipStream_t)stream);
}

size_t nc_ibi_onset_workspace_bytes(const nc_ctx* ctx, int n_files, int64_t total_frames) {
  (void)ctx;
  return nc::ibi_onset_ws_bytes(n_files, total_frames);
}

int nc_ibi_onset(nc_ctx* ctx, const float* sig, const int64_t* file_off, const int64_t* file_len, int n_files,
                 int64_t total_frames, int hop, float* onset_out, int64_t* frame_base_out, void* ws, size_t ws_bytes,
                 void* stream) {
  CHECK_CTX(ctx);
  SET_DEVICE(ctx);
  return nc::launch_ibi_onset(ctx->c, sig, file_off, file_len, n_files, total_frames, hop, onset_out,
                              frame_base_out, ws, ws_bytes, (hipStream_t)stream);
}

size_t nc_ibi_tempogram_workspace_bytes(const nc_ctx* ctx, int n_files, int64_t total_frames, int max_frames,
                                        int hop) {
  if (!ctx) return 0;
  return nc::ibi_tg_ws_bytes(ctx->c, n_files, total_frames, max_frames, hop);
}

int nc_ibi_tempogram(nc_ctx* ctx, const float* onset, const int64_t* frame_base, int n_files,
                     int64_t total_frames, int max_frames, int hop, double* tg_out, void* ws, size_t ws_bytes,
                     void* stream) {
  CHECK_CTX(ctx);
  SET_DEVICE(ctx);
  return nc::launch_ibi_tempogram(ctx->c, onset, frame_base, n_files, total_frames, max_frames, hop, tg_out, ws,
                                  ws_bytes, (hipStream_t)stream);
}

size_t nc_ibi_range_workspace_bytes(const nc_ctx* ctx, int n_files, int64_t total_rows) {
  (void)ctx;
  return nc::ibi_range_ws_bytes(n_files, total_rows);
}

int nc_ibi_mel_range(nc_ctx* ctx, const float* sig, const int64_t* file_off, const int64_t* file_len, int n_files,
                     const int64_t* t0, const int64_t* t1, int hop, int64_t total_rows, float* max_out, void* ws,
                     size_t ws_bytes, void* stream) {
  CHECK_CTX(ctx);
  SET_DEVICE(ctx);
  return nc::launch_ibi_mel_range(ctx->c, sig, file_off, file_len, n_files, t0, t1, hop, total_rows, max_out, ws,
                                  ws_bytes, (hipStream_t)stream);
}

int nc_ibi_onset_range(nc_ctx* ctx, int n_files, const int64_t* t0, int hop, int64_t total_out, const float* gmax,
                       float* onset_out, void* ws, int64_t total_rows, void* stream) {
  CHECK_CTX(ctx);
  SET_DEVICE(ctx);
  return nc::launch_ibi_onset_range(n_files, t0, hop, total_out, gmax, onset_out, ws, total_rows,
                                    (hipStream_t)stream);
}

int nc_ibi_tempogram_tiles(nc_ctx* ctx, const float* onset, const int64_t* frame_base, int n_files,
                           int64_t total_frames, int max_frames, int hop, const int64_t* b0, const int64_t* b1,
                           double* slab, void* ws, size_t ws_bytes, void* stream) {
  CHECK_CTX(ctx);
  SET_DEVICE(ctx);
  if (!b0 || !b1 || !slab) {
    nc::set_error("ibi_tempogram_tiles: b0, b1 and slab are required");
    return -2;
  }
  return nc::launch_ibi_tempogram_tiles(ctx->c, onset, frame_base, n_files, total_frames, max_frames, hop, b0, b1,
                                        slab, nullptr, ws, ws_bytes, (hipStream_t)stream);
}

int nc_ibi_tempogram_reduce(nc_ctx* ctx, const double* slab, const int64_t* frame_base, int n_files, int max_frames,
                            int hop, double* tg_out, void* stream) {
  CHECK_CTX(ctx);
  SET_DEVICE(ctx);
  return nc::launch_ibi_tempogram_reduce(ctx->c, slab, frame_base, n_files, max_frames, hop, tg_out,
                                         (hipStream_t)stream);
}

int nc_xcorr_search(nc_ctx* ctx, const float* sig, const int64_t* item_a, const int64_t* item_b, int n_items,
                    int win, double* dot, double* sqb, const int* w0, const int* w1, const int* win_self,
                    const int* cand0, const int* cand1, const int64_t* pa, const int64_t* pb, const int64_t* exp_pb,
                    int n_jobs, double* ratio_out, double* quality_out, void* stream) {
  CHECK_CTX(ctx);
  SET_DEVICE(ctx);
  return nc::launch_xcorr(sig, item_a, item_b, n_items, win, dot, sqb, w0, w1, win_self, cand0, cand1, pa, pb,
                          exp_pb, n_jobs, ratio_out, quality_out, (hipStream_t)stream);
}

size_t nc_align_workspace_bytes(const nc_ctx* ctx, int n_pairs, int n_speeds, int64_t total_len, int64_t max_len,
                                int max_offset_frames) {
  (void)ctx;
  return nc::align_ws_bytes(n_pairs, n_speeds, total_len, max_len, max_offset_frames);
}

int nc_align_offsets(nc_ctx* ctx, const float* sig, const int64_t* src_off, const int64_t* src_len,
                     const int64_t* nc_off, const int64_t* nc_len, int n_pairs, const double* speeds, int n_speeds,
                     int max_offset_frames, int64_t total_len, int64_t max_len, int* peak_out, int* speed_idx_out,
                     double* score_out, void* ws, size_t ws_bytes, void* stream) {
  CHECK_CTX(ctx);
  SET_DEVICE(ctx);
  return nc::launch_align_offsets(ctx->c, sig, src_off, src_len, nc_off, nc_len, n_pairs, speeds, n_speeds,
                                  max_offset_frames, total_len, max_len, peak_out, speed_idx_out, score_out, ws,
                                  ws_bytes, (hipStream_t)stream);
}

size_t nc_spectral_workspace_bytes(int64_t total_frames, int n_files, int64_t max_frames) {
  return nc::spectral_ws_bytes(total_frames, n_files, max_frames);
}

int nc_spectral_stats(nc_ctx* ctx, const float* sig, const int64_t* file_off, const int64_t* file_len,
                      const int64_t* frame_base, const double* bin_hz, const int* band_bins, int n_files,
                      int64_t total_frames, int64_t max_frames, float roll_percent, float* rms_out,
                      double* stats_out, double* bin_db_out, void* ws, size_t ws_bytes, void* stream) {
  CHECK_CTX(ctx);
  SET_DEVICE(ctx);
  return nc::launch_spectral(ctx->c, sig, file_off, file_len, frame_base, bin_hz, band_bins, n_files, total_frames,
                             max_frames, roll_percent, rms_out, stats_out, bin_db_out, ws, ws_bytes,
                             (hipStream_t)stream);
}

int nc_resample_poly(nc_ctx* ctx, const float* x, const int64_t* in_off, const int64_t* in_len, int n_files,
                     float* y, const int64_t* out_off, const int64_t* out_len, int64_t max_out, const double* h,
                     int h_len, int up, int down, int64_t pre_remove, void* stream) {
  CHECK_CTX(ctx);
  SET_DEVICE(ctx);
  return nc::launch_resample_poly(x, in_off, in_len, n_files, y, out_off, out_len, max_out, h, h_len, up, down,
                                  pre_remove, (hipStream_t)stream);
}

int nc_window_energy_blocks(nc_ctx* ctx, const float* sig, const void* trim_ws, int n_files, const int64_t* file_off,
                            const int64_t* win_off, const int* win_file, int n_win, int win_len, double* energy_out,
                            void* stream) {
  CHECK_CTX(ctx);
  SET_DEVICE(ctx);
  nc::MarkSpan ms_(ctx->c, "window_energy", (hipStream_t)stream);
  return nc::launch_window_energy_blocks(sig, trim_ws, n_files, file_off, win_off, win_file, n_win, win_len,
                                         energy_out, (hipStream_t)stream);
}

int nc_pcm16_to_f32(nc_ctx* ctx, const int16_t* x, int64_t n, float* y, void* stream) {
  CHECK_CTX(ctx);
  SET_DEVICE(ctx);
  return nc::launch_pcm16_to_f32(x, n, y, (hipStream_t)stream);
}

int nc_melodia_salience(nc_ctx* ctx, const float* sig, const int64_t* file_off, const int64_t* file_len,
                        const int64_t* frame_base, int n_files, int64_t total_frames, int hop, float sample_rate,
                        const float* win, int sal_min_bin, int* pk_count, int* pk_bin, float* pk_sal,
                        void* stream) {
  CHECK_CTX(ctx);
  SET_DEVICE(ctx);
  return nc::launch_melodia_salience(ctx->c, sig, file_off, file_len, frame_base, n_files, total_frames, hop,
                                     sample_rate, win, sal_min_bin, pk_count, pk_bin, pk_sal, (hipStream_t)stream);
}

}  // extern "C"
