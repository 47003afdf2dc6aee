#!/usr/bin/env python3
"""Which kernels run together in the pipelined config-3 step, untraced: Engine.analyze_batches
over K batches with every timed kernel recording its execution span (profile mode 2), the spans
dumped (nc_profile_dump_spans), and the time spent in each set of concurrently running kernels.
Only the timed (tagged) kernels record spans; the small ones (bootstraps, plans, gathers,
tails) count as "nothing", so the "-" row is an upper bound of the device idle.  With --marks
(profile mode 5) the small entry points get marker spans too (lower-case classes; each includes
its two one-thread marker launches), and "-" is the time nothing of the engine's runs.
    python3 tools/concurrency_spans.py [K] [--marks]"""
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "nightcore-to-flac-analyzer_amd"))

CLS = {"stft_mel": "S", "window_tg": "W", "tuning_peaks": "T", "decimate": "D", "cqt_low": "L", "cqt_high": "H",
       "tempo_beat": "B", "trim_blocks": "R", "tuning_select": "s",
       # marker spans (--marks): the small entry points
       "energy_gate": "g", "collect_valid": "v", "pitch_hz": "z", "tempo_prior": "r", "bootstrap": "b",
       "chroma_lag": "l", "chroma_plan": "p", "cqt_tail": "t", "window_energy": "e", "trim_bounds": "u"}


def table(spans, steps):
    ev = []
    for tag, a, b in spans:
        c = CLS.get(tag, "o")
        ev += [(a, 1, c), (b, -1, c)]
    ev.sort()
    active, acc, t_prev = {}, {}, ev[0][0]
    for t, d, c in ev:
        key = "".join(sorted(k for k, n in active.items() if n > 0)) or "-"
        acc[key] = acc.get(key, 0.0) + (t - t_prev)
        t_prev = t
        active[c] = active.get(c, 0) + d
    span = ev[-1][0] - ev[0][0]
    print(f"extent {span / steps:.3f} ms/step; " + ", ".join(f"{c}={k}" for k, c in CLS.items()))
    for k, v in sorted(acc.items(), key=lambda x: -x[1])[:20]:
        print(f"  {k:10s} {v / steps:7.3f} ms/step  {100 * v / span:5.1f} %")
    def frac(pred):
        return 100 * sum(v for k, v in acc.items() if pred(set(k))) / span
    print(f"stft_mel running {frac(lambda s: 'S' in s):.1f} %, a CQT kernel {frac(lambda s: bool(s & set('LH'))):.1f} %, "
          f"stft_mel with a CQT kernel {frac(lambda s: 'S' in s and bool(s & set('LH'))):.1f} %, "
          f"no large kernel {frac(lambda s: not (s & set('SWTDLH'))):.1f} %")


def gaps(spans, steps, top=12):
    """The largest intervals with no timed kernel running, with the kernels that end before and
    start after each (ms from the first span)."""
    iv = sorted((a, b, t) for t, a, b in spans)
    out, end, last = [], iv[0][1], iv[0][2]
    for a, b, t in iv[1:]:
        if a > end:
            out.append((a - end, end, last, t))
        if b > end:
            end, last = b, t
    tot = sum(g for g, *_ in out)
    print(f"gaps: {len(out)} totalling {tot / steps:.3f} ms/step; largest:")
    for g, at, before, after in sorted(out, reverse=True)[:top]:
        print(f"  {1e3 * g:8.1f} us at {at:9.3f} ms  after {before:14s} before {after}")


def main():
    import torch
    import bench
    from nightcore_analyzer import engine as E
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    K = int(args[0]) if args else 10
    mode = 5 if "--marks" in sys.argv else 2
    pairs = bench.make_pairs(64, 180.0, 1000, 16)
    eng = E.get_engine(0)
    sig = eng.upload_signals([a for nc, src in pairs for a in (nc, src)])
    p = E.Params(compute_ibi=False)
    eng.analyze_batches([sig] * K, p)
    eng.kernel_profile(mode)
    torch.cuda.synchronize()
    eng.analyze_batches([sig] * K, p)
    spans = eng.device_spans()
    eng.kernel_profile(0)
    table(spans, K)
    gaps(spans, K)
    if mode == 5:   # time per step in each small entry point (marker spans, summed)
        tot = {}
        for t, a, b in spans:
            if CLS.get(t, "o").islower() and t != "tuning_select":
                tot[t] = tot.get(t, 0.0) + (b - a)
        print("marker spans, ms per step:", {k: round(v / K, 3) for k, v in sorted(tot.items(), key=lambda x: -x[1])})


if __name__ == "__main__":
    main()
