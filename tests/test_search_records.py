"""Recorded default-Options searches on the engine (tools/run_search.py,
profiles/r0*_search_config*.json): every hall-of-fame loss the GPU run stored
is rechecked here on the CPU oracle, for the same trees and the same data
(BASELINE configs #1 and #4)."""
import json
from pathlib import Path

import numpy as np
import pytest

import oracle
import srhip

ROOT = Path(__file__).resolve().parent.parent
# every recorded search (r05_search_*, r05_final_search_*, r06_* ...): whatever DESIGN.md cites is rechecked
RECORDS = sorted((ROOT / "profiles").glob("r0*search_config*.json"))


def _data(cfg):
    if cfg == "config1":
        rng = np.random.default_rng(0)
        X = rng.standard_normal((5, 100)).astype(np.float32)
    else:
        rng = np.random.default_rng(41)
        X = rng.standard_normal((10, 100_000)).astype(np.float32)
    y = (np.float32(2) * np.cos(X[3]) + X[0] * X[0] - np.float32(2)).astype(np.float32)
    return X, y


@pytest.mark.parametrize("path", RECORDS, ids=[p.name for p in RECORDS])
def test_recorded_hall_of_fame_losses_match_the_oracle(path):
    rec = json.loads(path.read_text().splitlines()[-1])
    X, y = _data(rec["config"])
    f = rec["flat"]
    flat = srhip.FlatTrees(np.asarray(f["node_off"], np.int32), np.asarray(f["kind"], np.uint8),
                           np.asarray(f["arg"], np.uint16), np.asarray(f["const_off"], np.int32),
                           np.asarray(f["consts"], np.float32), np.diff(np.asarray(f["node_off"])))
    _, ref, ok = oracle.eval_loss_batch(flat, X, y, dtype=np.float32)
    stored = np.asarray([m["loss"] for m in rec["hall_of_fame"]])
    assert ok.all()
    np.testing.assert_allclose(stored, ref, rtol=1e-5)
    assert rec["niterations"] >= (40 if rec["config"] == "config1" else 2)
