"""Pre-tuned hipBLASLt / rocBLAS algorithm choice for the library GEMMs (forward + input-gradient
projections and the lm-head), via PyTorch TunableOp.

hipBLASLt's default heuristic leaves 5-25 % on the table for several Llama-150M shapes (e.g. the
q|k|v forward 197 -> 155 us, gate|up forward 320 -> 266 us, down dgrad 217 -> 195 us at 32k tokens;
``scripts/tune_gemms.py`` measures every candidate algorithm on the real shapes).  The winners are
shipped in-tree (``nanodiloco_amd/tuning/tunableop_gfx950.csv``); at start-up they are loaded with
tuning DISABLED, so no search ever runs inside a training / benchmark step, and shapes that are not
in the file keep the library default.  The file's validator lines pin the exact torch / HIP /
hipBLASLt / rocBLAS versions and the gfx950 arch: on any other stack TunableOp ignores it.
"""
from __future__ import annotations

import os

import torch

TUNING_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tuning")
DEFAULT_FILE = os.path.join(TUNING_DIR, "tunableop_gfx950.csv")

_enabled = False


def enable_tuned_gemms(device=None, path: str = DEFAULT_FILE) -> bool:
    """Load the pre-tuned GEMM table for this process (no-op off ROCm / off gfx950 / if disabled
    with ``NANODILOCO_TUNED_GEMM=0``).  Returns True when the table is active."""
    global _enabled
    if _enabled:
        return True
    if os.environ.get("NANODILOCO_TUNED_GEMM", "1") == "0" or not torch.cuda.is_available():
        return False
    if torch.version.hip is None or not os.path.exists(path):
        return False
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    if "gfx950" not in torch.cuda.get_device_properties(dev).gcnArchName:
        return False
    import torch.cuda.tunable as tunable
    tunable.enable(True)
    tunable.tuning_enable(False)
    tunable.record_untuned_enable(False)
    # results are read from the shipped table; anything TunableOp would write goes to /tmp
    tunable.set_filename(os.path.join(os.environ.get("TMPDIR", "/tmp"), f"nd_tunableop_{os.getpid()}.csv"))
    ok = tunable.read_file(path)
    _enabled = bool(ok)
    if not ok:
        tunable.enable(False)
    return _enabled
