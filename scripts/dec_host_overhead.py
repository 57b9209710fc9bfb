import sys, time, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch, clay_amd
from clay_amd import ClayCode
c = ClayCode(10, 4, 13)
chunk = c.encoded_chunk_size(1 << 30)
full = torch.randint(0, 256, (c.n, chunk), dtype=torch.uint8, device="cuda")
outs = torch.zeros((c.n, chunk), dtype=torch.uint8, device="cuda")
for st, er in ((torch.cuda.current_stream(), [0]), (torch.cuda.Stream(), [0]), (torch.cuda.current_stream(), [0, 4, 8, 12]), (torch.cuda.Stream(), [0, 4, 8, 12])):
    ins = [None if i in er else full[i] for i in range(c.n)]
    ous = [outs[i] if i in er else None for i in range(c.n)]
    fn = lambda: c.decode_device(ins, er, ous, chunk, 0, st.cuda_stream)
    for _ in range(50): fn()
    torch.cuda.synchronize()
    # host time per call (no sync)
    t0 = time.perf_counter(); n = 30
    for _ in range(n): fn()
    t1 = time.perf_counter(); torch.cuda.synchronize()
    host_us = (t1 - t0) / n * 1e6
    # batch events
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(n): fn()
    e1.record(st); torch.cuda.synchronize()
    batch = e0.elapsed_time(e1) / n
    # per-call events
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in evs:
        a.record(st); fn(); b.record(st)
    torch.cuda.synchronize()
    per = sorted(a.elapsed_time(b) for a, b in evs)
    print(er, "default" if st.cuda_stream == 0 else "own stream", clay_amd.last_exec_path(), "host us/call %.1f" % host_us, "batch ms %.4f" % batch, "per-call median ms %.4f" % per[n // 2], flush=True)
