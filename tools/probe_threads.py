"""Probe: does the HIP transport leave threads behind?  Counts this process's OS threads
(/proc/self/task) across 20 comms that defer delayed launches to the host timer and are
shut down and closed, then 5 that are only dropped (garbage-collected).  r04: 18 threads at
the start and after every stage -- the timer threads are joined at close (profiles/
r04_gated_stall.txt).  Usage (GPU box): python tools/probe_threads.py"""
import os, sys
sys.path[:0] = ['mpistragglers.jl_amd']
import torch
import mpiasyncpools as M
def nt():
    return len(os.listdir('/proc/self/task'))
torch.zeros(1, device='cuda')
print('start', nt(), flush=True)
for i in range(20):
    c = M.DeviceComm(3)
    for r in range(1, 4):
        c.set_task(r, 'kmap2')
        c.set_delays(r, [1_000_000])
    p = M.MPIAsyncPool(3)
    s = torch.zeros(1, dtype=torch.float64, device='cuda')
    rb = torch.zeros(9, dtype=torch.float64, device='cuda')
    M.asyncmap_(p, s, rb, torch.zeros(3, dtype=torch.float64, device='cuda'), torch.zeros_like(rb), c, nwait=3)
    c.shutdown()
    c.close()
    if i in (0, 1, 4, 19):
        print('after', i + 1, 'comms', nt(), flush=True)
for i in range(5):  # comms never shut down or closed explicitly (garbage)
    c = M.DeviceComm(3)
    for r in range(1, 4):
        c.set_task(r, 'kmap2')
        c.set_delays(r, [1_000_000])
    p = M.MPIAsyncPool(3)
    M.asyncmap_(p, s, rb, torch.zeros(3, dtype=torch.float64, device='cuda'), torch.zeros_like(rb), c, nwait=3)
    del c, p
import gc; gc.collect()
print('after 5 dropped comms', nt(), flush=True)
