"""Seeded inputs of the MSF-evaluation parity case (TEST INFRASTRUCTURE).

Shared by the fixture generator (oracle/gen_golden.py gen_msf: the reference's evaluate_msf,
val_mm.py:87-120) and the GPU test (tests/test_gpu_drivers.py::test_evaluate_msf_matches_reference)
so both build bit-identical inputs from the seeds.  Scales and flip are configs/nyu_rgbd.yaml's
EVAL.MSF settings; the model is the tiny fp32 CMNeXt of the cmnext_tiny fixture.
"""
import numpy as np

from fill import seeded

MSF_CASE = dict(B=2, H=96, W=128, n_cls=5, fill_seed=29, input_seed=300,
                scales=(0.5, 0.75, 1.0, 1.25, 1.5, 1.75), flip=True)


def msf_inputs():
    c = MSF_CASE
    rgb = seeded((c["B"], 3, c["H"], c["W"]), c["input_seed"])
    dep = seeded((c["B"], 3, c["H"], c["W"]), c["input_seed"] + 1, "uniform")
    lbl = (seeded((c["B"], c["H"], c["W"]), c["input_seed"] + 2, "uniform") * c["n_cls"]).astype(np.int64)
    lbl = lbl.clip(0, c["n_cls"] - 1)
    lbl[seeded((c["B"], c["H"], c["W"]), c["input_seed"] + 3, "uniform") < 0.1] = 255
    return rgb, dep, lbl
