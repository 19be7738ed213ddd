import time, os, sys, numpy as np
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from nmfconsensus_amd.nmf import cophenetic_batch
rng=np.random.default_rng(0)
def cons_stack(n, ks, R):
    out=[]
    for k in ks:
        lab=rng.integers(0,k,(R,n)).astype(np.int8)
        c=np.zeros((n,n))
        for r in range(R): c+= (lab[r][:,None]==lab[r][None,:])
        out.append(c/R)
    return np.stack(out)
C3=cons_stack(500, range(2,11), 200)
cophenetic_batch(C3, symmetric=True)
for _ in range(3):
    t=time.perf_counter(); cophenetic_batch(C3, symmetric=True); print('C3 cophenetic 9 x 500:', round((time.perf_counter()-t)*1e3,1),'ms', flush=True)
print('cpus', os.cpu_count(), len(os.sched_getaffinity(0)))
