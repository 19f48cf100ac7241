"""Achieved-parity record of the GPU parity tests.

compare_forward / compare_backward (tests/test_gpu_parity.py) record, per test case, the measured errors of the HIP
path against the oracle: integer mismatches (always 0 when they pass), threshold-flip candidate counts, colour /
inverse-depth maxima inside and outside the flip candidates, and per-gradient relative L2 over all Gaussians and over
the Gaussians no flip candidate touches.  With GSR_PARITY_JSON=<path> set, tests/conftest.py writes the record there
at the end of the session (profiles/parity_r3.json is one such run), so the bars in the tests can be checked against
what is actually achieved.
"""
from __future__ import annotations

import json
import os

RECORD: dict = {}


def record(case: str, kind: str, data: dict) -> None:
    RECORD.setdefault(case, {})[kind] = data
    dump()  # after every case, so a run cut short still leaves its record


def dump() -> None:
    path = os.environ.get("GSR_PARITY_JSON")
    if not path or not RECORD:
        return
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "w") as f:
        json.dump(RECORD, f, indent=1, sort_keys=True)
