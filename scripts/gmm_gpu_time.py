"""Generator throughput: host numpy restatement (gmm.gmm_pair) vs the device generator in
exact mode (reference streams) and device mode (Philox), N = 1000 two-layer graphs."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mdcommunity_amd import gmm, gmm_gpu  # noqa: E402

G = int(sys.argv[1]) if len(sys.argv) > 1 else 256
gmm_gpu.gmm_pairs(1000, [0], exact=False)  # warm (module load, first launch)
t = time.perf_counter()
for s in range(16):
    gmm.gmm_pair(1000, seed=s)
host = (time.perf_counter() - t) / 16
t = time.perf_counter()
gmm_gpu.gmm_pairs(1000, range(64), exact=True)
ex = (time.perf_counter() - t) / 64
t = time.perf_counter()
gmm_gpu.gmm_pairs(1000, range(G), exact=False)
dv = (time.perf_counter() - t) / G
print(f"N=1000 two-layer GMM graph: host numpy {host * 1e3:.1f} ms, device exact {ex * 1e3:.1f} ms, "
      f"device Philox {dv * 1e3:.2f} ms per graph ({G} graphs)", flush=True)
