"""Prints the SHA-256 of the synthetic C3 matrix (planted_matrix(20000, 500)) on this host: the C3 golden
(tests/golden/golden_c3.npz) records the one it was generated from, and the GPU test refuses another."""
import hashlib, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from nmfconsensus_amd.synthetic import planted_matrix
A = planted_matrix(20000, 500)
print(hashlib.sha256(np.ascontiguousarray(A).tobytes(order="F")).hexdigest())
