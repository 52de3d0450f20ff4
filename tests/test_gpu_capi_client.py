"""The C ABI from a plain C process (tests/c/capi_client.c): the system ROCm runtime and
hipMalloc buffers of exactly the sizes the ABI states, as a Julia `ccall` user has them.

torch's caching allocator leaves slack around small tensors, so the Python-driven tests
could not see a kernel reading past its buffers; this client did: lsq_grad_kernel's clamp
for 16-B vectors past `cols` (lanes of the last vector group when cols < 64 vectors) pointed
at vector `lane` of the row instead of vector 0, past the end of A on the last row (fixed in
lsq_kernel.hip / lsqw_kernel.hip).  Cases: narrow rows with a partial vector group (fp64 64
columns, fp32 100 and 8), a full-width narrow row, wide rows with a one-vector last slice;
1-3 workers; the batched bf16 variant (lsqp4: a ragged last block, a wave with one
32-column strip, 32 and 2048 columns; the two-pass kernels at 2080 and 4096 columns); every
reply against a host fp64 gradient of the device's own inputs (relative 1e-12 fp64, 1e-5
fp32 / bf16-in-fp32: BASELINE's tolerances).  Beyond one call: mpa_lsq_descent (fused tail,
launch-ahead; the epoch kernel for wide rows) and mpa_lsqb_descent for several epochs against
a host fp64 replay, and a k-of-n run under a gated schedule with a stale harvest in the wait
loop, its held re-dispatch, a phase-1 harvest, a tie and waitall!."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLIENT = os.path.join(ROOT, "mpistragglers.jl_amd", "_build", "capi_client")

pytestmark = pytest.mark.gpu


def test_c_client_of_the_abi(built):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    assert os.path.exists(CLIENT), "build() builds tests/c/capi_client"
    out = subprocess.run([CLIENT], capture_output=True, text=True, timeout=120)
    print(out.stdout)
    assert out.returncode == 0, (out.stdout[-2000:], out.stderr[-2000:])
    lines = [ln.split() for ln in out.stdout.splitlines() if ln.startswith("case ")]
    assert len(lines) == 19 and out.stdout.rstrip().endswith("ok")
    for ln in lines:
        dtype, err = ln[1], float(ln[6])
        assert err <= (1e-12 if dtype == "f64" else 1e-5), ln
