// nc_capi.cpp — extern "C" entry points of libncgpu.so (declared in include/ncgpu.h).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>

#include "../../include/ncgpu.h"
#include "nc_engine.h"

namespace nc {

thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }

// kernels (defined in the .hip translation units)
struct BeatArgs;
size_t window_stage_ws_bytes(const Context& ctx, int n_win, int T);
int launch_window_stage(Context& ctx, const float* sig, const int64_t* win_off, const uint8_t* active,
                        int n_win, int win_len, int hop, float* onset_out, double* tg_out,
                        double* energy_out, void* ws, size_t ws_bytes, hipStream_t st);
int launch_tempo_beats_c(Context& ctx, const float* onset, const int64_t* off, const int* len, int n_seq,
                         int max_len, const double* tg, int acw, const double* start_bpm,
                         const int* prior_idx, const uint8_t* active, int hop, int trim, double* bpm_out,
                         int* lag_out, int* nbeats_out, double* margin_out, int* beats_out,
                         int64_t total_frames, void* ws, size_t ws_bytes, hipStream_t st);
int launch_nc_prior(const double* bpm, const int* nbeats, const uint8_t* active, const int* src_w0,
                    const int* src_w1, const int64_t* src_len, const int64_t* nc_len, int n_pairs,
                    double* prior_out, hipStream_t st);
int launch_ibi_from_beats(const int* beats, const int64_t* off, const int* nbeats, int n_seq, int hop,
                          int min_ibis, double* ibi_out, int* n_ibi, hipStream_t st);
size_t trim_ws_bytes(const int64_t* host_file_len, int n_files);
int launch_trim(Context& ctx, const float* sig, const int64_t* file_off, const int64_t* file_len, int n_files,
                int64_t max_frames, float top_db, int64_t* out_start, int64_t* out_end, void* ws,
                size_t ws_bytes, hipStream_t st);

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

int nc_create(int device, nc_ctx** out) {
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
  nc_ctx* c = new nc_ctx();
  c->c.device = device;
  int cu = 0;
  if (hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cu > 0)
    c->c.num_cu = cu;
  nc::build_tables(c->c);
  if (!c->c.t.tw4096 || !c->c.t.cqt_w || !c->c.t.halfband) {
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
  nc::free_tables(ctx->c);
  delete ctx;
  return 0;
}

int nc_num_cu(const nc_ctx* ctx) { return ctx ? ctx->c.num_cu : -1; }

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
                                 energy_out, ws, ws_bytes, (hipStream_t)stream);
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
  return nc::launch_nc_prior(bpm, nbeats, active, src_w0, src_w1, src_len, nc_len, n_pairs, prior_out,
                             (hipStream_t)stream);
}

int nc_ibi_from_beats(nc_ctx* ctx, const int* beats, const int64_t* off, const int* nbeats, int n_seq, int hop,
                      int min_ibis, double* ibi_out, int* n_ibi, void* stream) {
  CHECK_CTX(ctx);
  SET_DEVICE(ctx);
  return nc::launch_ibi_from_beats(beats, off, nbeats, n_seq, hop, min_ibis, ibi_out, n_ibi,
                                   (hipStream_t)stream);
}

}  // extern "C"
