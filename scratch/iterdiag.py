import sys, time, json, numpy as np
sys.path.insert(0,'planning-motion_planning_amd')
import torch
import eikonal
from eikonal import terrain, _lib as L
dev=torch.device("cuda",0)
N=int(sys.argv[1]) if len(sys.argv)>1 else 4096
cost=terrain.cost_block(0,0,N,N,N,N,seed=42,device=dev).contiguous()
T=torch.empty_like(cost)
s=torch.cuda.current_stream(dev).cuda_stream
ctx=eikonal.Context(0)
fim=eikonal.Fim2d(ctx,1,N,N,L.EIK_F32)
for rounds in (1,2,3):
    ctx.set_option(L.OPT_MAX_ROUNDS, rounds)
    for rep in range(2):
        ctx.set_option(L.OPT_TIMING,1)
        fim.start(cost.data_ptr(),T.data_ptr(),[(N//2,N//2)],s)
        rows=[]; prev=0.0
        while True:
            a=fim.iterate(1); st=fim.stats()
            rows.append((a, st["sweep_ms"]-prev)); prev=st["sweep_ms"]
            if a==0: break
        st=fim.stats()
        ctx.set_option(L.OPT_TIMING,0)
        torch.cuda.synchronize(); t0=time.perf_counter(); fim.solve(cost.data_ptr(),T.data_ptr(),[(N//2,N//2)],s); torch.cuda.synchronize(); el=(time.perf_counter()-t0)*1e3
        st2=fim.stats()
        print(f"rounds={rounds} rep={rep} iters={st['iterations']} visits={st['tile_visits']} sweep_ms={st['sweep_ms']:.3f} | solve wall {el:.3f} ms iters {st2['iterations']} visits {st2['tile_visits']}", flush=True)
        if rep==0:
            act=[r[0] for r in rows]; us=[round(r[1]*1e3,1) for r in rows]
            print("  active per iter:", act[:120], flush=True)
            print("  us per launch:", us[:120], flush=True)
