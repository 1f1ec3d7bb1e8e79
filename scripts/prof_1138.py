import os, sys, torch
sys.path.insert(0, os.getcwd())
import sparsecholesky_amd as sc
A = sc.load_matrix_market_to_csc("tests/golden/1138_bus.mtx")
s = sc.Symbolic(A, use_graph=0)
num = sc.Numeric(s, device=0)
d = torch.from_numpy(A.x).to("cuda:0")
for _ in range(30): num.factor_device(d.data_ptr(), sync=True)
