// nc_engine.h — internal (C++) interface between the C-ABI layer and the HIP
// kernels.  Not part of the public boundary (that is include/ncgpu.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

namespace nc {

constexpr int kSR = 22050;
constexpr int kNFFT = 2048;     // STFT / mel frame (onset_strength, piptrack)
constexpr int kNMels = 128;
constexpr int kCqtBins = 252;   // 7 octaves x 36
constexpr int kCqtBpo = 36;
constexpr int kCqtFilt = 36;    // filters per octave
constexpr int kCqtNfft = 1024;
constexpr int kNTunings = 100;  // tuning grid (-0.50 .. 0.49 step 0.01)
constexpr int kHalfbandK = 23;  // decimator half length (47 taps)

// Device-resident constant tables, built once per context (double precision on
// the host, rounded to f32).
struct Tables {
  float2* tw = nullptr;         // exp(-2 pi i m / 8192)
  float* hann2048 = nullptr;    // periodic Hann, STFT window
  float* hann_ac512 = nullptr;  // periodic Hann(344): tempogram window at hop 512
  float* hann_ac64 = nullptr;   // periodic Hann(2756): tempogram window at hop 64
  int ac512 = 0, ac64 = 0;
  double* wsq512 = nullptr;     // hann_ac512[j]^2 in f64 (lag-0 autocorrelation, the tempogram normaliser)
  double* wsq64 = nullptr;      // hann_ac64[j]^2 in f64
  // Slaney mel filterbank (sr 22050, n_fft 2048, 128 bands, fmax 11025) in CSR
  int* mel_lo = nullptr;
  int* mel_len = nullptr;
  int* mel_off = nullptr;
  float* mel_w = nullptr;
  int mel_nnz = 0;
  // the same filterbank as two lane slots (slot 0: bands 0..63, slot 1: bands 64..127, lane
  // l of slot s holds band mel_band[64 s + l]), each read from a 16-byte aligned first bin
  // lo4 in float4 steps: weights [mel_j0 + mel_j1][64] float4 (zero outside the band), lo4 /
  // steps per (slot, lane)
  float4* mel_w4 = nullptr;
  int* mel_lo4 = nullptr;  // [2][64]
  int* mel_nj4 = nullptr;  // [2][64]
  int* mel_band = nullptr;  // [2][64]
  int mel_j0 = 0, mel_j1 = 0;
  int mel_reach = 0;  // 1 + the largest power index the unrolled mel steps read (lo4 + 4 J)
  // CQT: per tuning index, per filter: [lo, len, off] into a complex weight pool
  int* cqt_lo = nullptr;        // [kNTunings][36]
  int* cqt_len = nullptr;
  int* cqt_off = nullptr;
  float2* cqt_w = nullptr;      // sparse basis rows (octave-0 basis, sqrt(sr/my_sr) applied per octave)
  float* cqt_inv_sqrt_len = nullptr;  // [kNTunings][252]  1/sqrt(lengths)
  int cqt_maxlen = 0;
  int cqt_maxnnz = 0;           // max over tunings of the 36 rows' total length
  double* halfband = nullptr;   // 2K+1 taps
  float halfband_f32[2 * kHalfbandK + 1] = {};  // host copy, rounded to f32 (decimate3 kernel argument)
  // MFMA CQT (cqt_mfma_kernel): the 36 rows as 1024-tap time-domain filters, split into f16
  // hi + lo at a per-filter power-of-two scale, in 16x16x32 B-fragment order
  // [tuning][k-step 32][n-tile 5][hi, lo][lane 64] x 8 halves (nc_tables.cpp)
  uint4* cqm_b = nullptr;
  int* cqm_bexp = nullptr;      // [kNTunings][36] filter scale exponents
  float cqm_gpow[7] = {};       // bound of max|octave o| / max|octave 0|: (sqrt(2) sum|h|)^o, rounded up
};

struct KernelTimers;  // nc_prof.cpp

struct Context {
  int device = 0;
  int num_cu = 256;
  // persistent grids of the window chain's STFT and the chroma chain's tuning FFT (0: num_cu).
  // Measurement knobs (NC_STFT_CUS / NC_CHROMA_CUS at nc_create) for CU-masked streams: a
  // persistent kernel sized to the CUs its stream may use (round 6)
  int stft_cus = 0, chroma_cus = 0;
  // sample rate the rate-dependent tables are built for (nc_create_rate, ABI 5): the mel
  // filterbank and the tempogram windows (tempo.py:27-173 at any sr); the CQT / tuning / trim
  // tables stay at kSR and their entry points need sr == kSR
  int sr = kSR;

  hipStream_t stream = nullptr;
  Tables t;
  KernelTimers* timers = nullptr;  // non-null while per-kernel profiling is enabled
};

// Profile mode 5 only: a span for a small entry point whose kernels record none themselves,
// made by two one-thread marker launches on its stream around them (the first records the
// wall clock when the stream reaches it, the second after the kernels): the span includes the
// markers' own dispatch, so it is an upper bound.  No-op in every other mode.
class MarkSpan {
 public:
  MarkSpan(Context& ctx, const char* tag, hipStream_t st);
  ~MarkSpan();
  MarkSpan(const MarkSpan&) = delete;
  MarkSpan& operator=(const MarkSpan&) = delete;

 private:
  unsigned long long* span_ = nullptr;
  hipStream_t st_;
};
int launch_span_mark(unsigned long long* span, int end, hipStream_t st);

// Brackets one kernel launch with HIP events on its stream when profiling is enabled
// (nc_profile_enable); no-op otherwise.  Used to time the dominant kernels live.
class KTimer {
 public:
  KTimer(Context& ctx, const char* tag, hipStream_t st);
  ~KTimer();
  KTimer(const KTimer&) = delete;
  KTimer& operator=(const KTimer&) = delete;
  // device span slot of this launch (nc_device.h Span / span_record), or null
  unsigned long long* span() const { return span_; }

 private:
  unsigned long long* span_ = nullptr;
  Context& ctx_;
  const char* tag_;
  hipStream_t st_;
  void* stop_ = nullptr;
};
void free_timers(Context& ctx);
void profile_enable(Context& ctx, int mode);
int profile_read(Context& ctx, const char* tag, double* total_ms, int* launches);
int profile_read_span(Context& ctx, const char* tag, double* total_ms, int* launches);
int profile_read_busy(Context& ctx, double* busy_ms, double* extent_ms, int* launches);
int profile_dump_spans(Context& ctx, char* tags, int tags_cap, int* tag_index, double* start_ms, double* end_ms,
                       int cap, int* n);

// bootstrap.hip job description (see nc_bootstrap_ratio in include/ncgpu.h)
struct BootArgs {
  const double* values;
  const int64_t* a_off;
  const int* a_n;
  const int64_t* b_off;  // nullable
  const int* b_n;        // nullable
  int n_boot;
  const uint64_t* seed;  // [job][4] = state_hi, state_lo, inc_hi, inc_lo
  double idx_lo, g_lo, idx_hi, g_hi;
  double* point_out;
  double* lo_out;
  double* hi_out;
  double* boot_out;      // nullable [job][n_boot]
  const int64_t* ws_off; // [job] byte offsets into ws
  const int* cap;        // [job] capacity (>= a_n + b_n)
  char* ws;
  int min_n;             // jobs with a_n < min_n (or b_n < min_n when B is present) are skipped
};

void build_tables(Context& ctx);
void free_tables(Context& ctx);

// error plumbing (thread-local message, int status)
void set_error(const std::string& msg);

}  // namespace nc

// timing probe (tools/var_build.sh variants only): bit k launches kernel k twice (the kernels
// listed are idempotent), so the step's growth is that launch's cost inside the pipeline.
// 1 tempo_beat<256, true>, 2 bootstrap_finish, 4 window_tg, 8 decimate3 (both launches),
// 16 cqt_mfma_low, 32 cqt_mfma (octaves 3-6); tools/twice_probe.sh, profiles/r5_twice_probe.txt
#ifndef NC_PROBE_TWICE
#define NC_PROBE_TWICE 0
#endif
#define NC_PROBE_REPS(k) (1 + ((NC_PROBE_TWICE >> (k)) & 1))
#define NC_HIP(call)                                                                  \
  do {                                                                                \
    hipError_t _e = (call);                                                           \
    if (_e != hipSuccess) {                                                           \
      nc::set_error(std::string(#call) + ": " + hipGetErrorString(_e));              \
      return -1;                                                                      \
    }                                                                                 \
  } while (0)
