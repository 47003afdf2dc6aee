import sys, time
sys.path[:0] = ['/root/repo', '/root/repo/nightcore-to-flac-analyzer_amd']
import numpy as np, torch
from nightcore_analyzer import engine as E
eng = E.get_engine(0)
rng = np.random.default_rng(0)
jobs = [(rng.random(60) * 50 + 100, rng.random(70) * 50 + 100) for _ in range(200)]
for _ in range(3): eng.bootstrap(jobs, seed=42)
torch.cuda.synchronize(); t = time.perf_counter()
for _ in range(20): r = eng.bootstrap(jobs, seed=42)
torch.cuda.synchronize(); print("bootstrap 200 jobs ms/call", (time.perf_counter() - t) / 20 * 1e3)
print(r[0], r[-1])
