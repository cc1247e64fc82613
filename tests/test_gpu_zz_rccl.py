"""The RCCL-backed overlapped gradient exchange of irads/graph_step.py, in a child process and in
the last file of the GPU suite (zz): a communicator's background threads then never share a
process with the other GPU tests.  Two suite runs aborted without a message in this test's RCCL
section when it ran in the pytest process; the child's whole output is kept in
$IRADS_REPORT_DIR/rccl_overlap_worker.log (default gpurun_out/)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_graph_step_overlapped_exchange_capture():
    """comm="overlap": the bucketed all-reduces are issued from post-accumulate-grad hooks on a side
    stream and captured into the graph with the backward and AdamW.  On a 1-rank RCCL group (the
    collective is the identity) gradients and updated parameters equal the un-bucketed graph
    step's (up to MIOpen's non-reproducible fuse_q convolution solvers), so the hooks, the
    flat-buffer pack / unpack and the capture of the RCCL calls are exercised
    (tests/_rccl_overlap_worker.py); the 2-rank averaging is test_dp_two_ranks_gradients."""
    env = dict(os.environ)
    env.setdefault("NCCL_DEBUG", "WARN")
    env["TORCH_SHOW_CPP_STACKTRACES"] = "1"
    port = str(29700 + os.getpid() % 200)
    p = subprocess.Popen([sys.executable, "-X", "faulthandler", os.path.join(ROOT, "tests", "_rccl_overlap_worker.py"),
                          port], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    try:
        out = p.communicate(timeout=150)[0].decode(errors="replace")
    finally:
        if p.poll() is None:  # our own child only
            p.kill()
            p.wait()
    log_dir = os.environ.get("IRADS_REPORT_DIR", os.path.join(ROOT, "gpurun_out"))
    os.makedirs(log_dir, exist_ok=True)
    with open(os.path.join(log_dir, "rccl_overlap_worker.log"), "w") as f:  # the whole child output
        f.write(out)
    errs = [ln for ln in out.splitlines() if "error" in ln.lower() and "Traceback" not in ln][:8]
    assert p.returncode == 0 and "OK rel" in out, (p.returncode, errs, out[-3000:])
