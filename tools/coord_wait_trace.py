"""Where the coordinator's kernels wait: from a `rocprofv3 --kernel-trace --hip-runtime-trace` run
of bench.py (DIR holds <cfg>_kernel_trace.csv and <cfg>_hip_api_trace.csv), per epoch / exchange
kernel: its host launch call, launch-call end -> kernel start, its duration, and how many
lsq_grad_kernel tasks were running at the call and during the kernel
(profiles/r05_null_stream.txt).

    python tools/coord_wait_trace.py gpurun_out/<tag>/rt
"""
import csv
import glob
import sys
d=sys.argv[1]
api=list(csv.DictReader(open(glob.glob(d+'/*_hip_api_trace.csv')[0])))
ker=list(csv.DictReader(open(glob.glob(d+'/*_kernel_trace.csv')[0])))
for r in api+ker:
    r['s']=int(r['Start_Timestamp']); r['e']=int(r['End_Timestamp'])
bycorr={r['Correlation_Id']:r for r in api}
def nm(k):
    for t in ('epoch_kernel','lsq_grad_kernel','exchange_kernel','generate_kernel','read_peak'):
        if t in k: return t
    return 'other'
for k in ker: k['n']=nm(k['Kernel_Name'])
ker.sort(key=lambda r:r['s'])
lsq=[k for k in ker if k['n']=='lsq_grad_kernel']
for k in ker:
    if k['n'] not in ('epoch_kernel','exchange_kernel'): continue
    L=bycorr.get(k['Correlation_Id'])
    if not L or k['s']<lsq[0]['s']: continue
    run_call=sum(1 for l in lsq if l['s']<L['e']<l['e'])
    run_exec=sum(1 for l in lsq if l['s']<k['e'] and l['e']>k['s'])
    started=sum(1 for l in lsq if L['e']<l['s']<k['s'])
    print('%-15s q%s call %5.1f us, call end->start %6.1f us, dur %5.1f us, lsq running at call %d / during exec %d, lsq started in between %d'%(k['n'],k['Queue_Id'],(L['e']-L['s'])/1e3,(k['s']-L['e'])/1e3,(k['e']-k['s'])/1e3,run_call,run_exec,started))
