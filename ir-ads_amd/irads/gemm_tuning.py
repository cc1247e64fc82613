"""hipBLASLt kernel selection for the step's library GEMMs (PyTorch TunableOp).

The dense projections (qkv / proj / fc1 / fc2 of the Swin trunk, the head and fusion
Linears) stay on hipBLASLt, but its default heuristic pick is far from the best kernel for
several of the step's shapes (tall-skinny M = 2^17 tokens x K = 128 at stage 0, reported at
~300 TF/s).  TunableOp benchmarks the hipBLASLt / rocBLAS solutions for each (op, shape,
dtype) once and records the winner; the table produced on an MI355X
(scripts/tune_gemms.py) ships in tuned/ and is loaded read-only here, so a run selects the
tuned kernels without tuning anything.  Without the table nothing changes.
"""
import os

import torch

TUNED_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuned")
TABLE = os.environ.get("IRADS_GEMM_TABLE", os.path.join(TUNED_DIR, "tunableop_mi355x0.csv"))


def use_tuned_gemms(table=TABLE):
    """Enable TunableOp in lookup-only mode with the shipped table; returns True if loaded."""
    if not (os.path.exists(table) and torch.cuda.is_available()):
        return False
    t = torch.cuda.tunable
    t.enable(True)
    t.tuning_enable(False)
    t.record_untuned_enable(False)
    t.set_filename(table)  # every rank reads the same table (identical GPUs)
    return bool(t.read_file(table))


def start_tuning(out_file, max_ms=30):
    """Tuning mode: every new GEMM shape is benchmarked (up to max_ms per shape) and recorded."""
    t = torch.cuda.tunable
    t.enable(True)
    t.tuning_enable(True)
    t.set_max_tuning_duration(max_ms)
    t.set_filename(out_file)
