import sys, json
sys.path.insert(0, "tools"); sys.path.insert(0, ".")
import torch
from bench_gemm import run
for s in [(16384,16384,16384,0,1,False,0.0,{}), (16384,16384,16384,0,0,False,0.0,{}),
          (16384,16384,16384,1,0,False,0.0,{}), (16384,16384,16384,1,1,False,0.0,{}),
          (16384,16384,16384,0,0,False,0.0,{"tri_b":True}), (16384,16384,16384,0,0,False,0.0,{"tri_a":True}),
          (16384,16384,16384,0,1,False,0.0,{"tri_b":True})]:
    m,n,k,ta,tb,lo,beta,kw = s
    print(json.dumps(run(m,n,k,ta,tb,lo,beta,reps=3,**kw)), flush=True)
