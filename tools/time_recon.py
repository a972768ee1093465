"""Wall time of run_sankoff(..., return_path=True) at the C2 shape (64 taxa x 10 000 sites x 4), host API end to end."""
import sys, time
sys.path.insert(0, '.')
import numpy as np, torch
from trex_amd import run_sankoff
from trex_amd.topology import create_balanced_binary_tree
nl, L, Q = 64, 10000, 4
A = create_balanced_binary_tree(nl)
rng = np.random.default_rng(0)
seqs = rng.integers(0, Q, size=(nl, L))
C = (np.ones((Q, Q)) - np.eye(Q)).astype(np.float32)
for _ in range(3):
    out = run_sankoff(A, C, seqs, 2 * nl - 1, Q, nl, return_path=True)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    out = run_sankoff(A, C, seqs, 2 * nl - 1, Q, nl, return_path=True)
torch.cuda.synchronize()
print("run_sankoff(return_path) C2 shape ms:", (time.perf_counter() - t0) / 20 * 1e3)
