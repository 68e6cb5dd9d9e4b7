"""The pvsim / metersim entry points (tmhpvsim_amd/cli.py): the reference's
options (pvsim.py:103-121, metersim.py:79-95), the batched offline mode and its
output formats (the CSV of pvsim.py:72-84, the messages of metersim.py:38-42)."""
import csv
import json

import numpy as np
import pytest
from click.testing import CliRunner

from tmhpvsim_amd.cli import main


def _gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def test_reference_options_are_accepted():
    r = CliRunner().invoke(main, ["pvsim", "--help"])
    assert r.exit_code == 0
    for opt in ("--amqp-url", "--exchange", "--verbose", "--realtime / --no-realtime", "--batch"):
        assert opt in r.output
    r = CliRunner().invoke(main, ["metersim", "--help"])
    assert r.exit_code == 0 and "--no-realtime" in r.output


def test_amqp_pipeline_is_out_of_scope_and_says_so(tmp_path):
    r = CliRunner().invoke(main, ["pvsim", str(tmp_path / "x.csv"), "--no-realtime"])
    assert r.exit_code != 0 and "--batch" in r.output


def test_batch_needs_no_realtime(tmp_path):
    r = CliRunner().invoke(main, ["pvsim", str(tmp_path / "x.csv"), "--batch", "2"])
    assert r.exit_code != 0 and "--no-realtime" in r.output


@pytest.mark.skipif(_gpu(), reason="CPU-only check")
def test_batch_has_no_cpu_fallback(tmp_path):
    r = CliRunner().invoke(main, ["pvsim", str(tmp_path / "x.csv"), "--batch", "2", "--no-realtime",
                                  "--seconds", "60"])
    assert r.exit_code != 0 and "no GPU" in r.output


@pytest.mark.gpu
def test_pvsim_batch_writes_reference_csv(tmp_path):
    f = tmp_path / "pv.csv"
    npz = tmp_path / "all.npz"
    r = CliRunner().invoke(main, ["pvsim", str(f), "--batch", "8", "--no-realtime", "--start", "2019-09-06T12:00:00",
                                  "--seconds", "600", "--all-chains", str(npz)])
    assert r.exit_code == 0, r.output
    rows = list(csv.reader(open(f)))
    assert rows[0] == ["time", "meter", "pv", "residual load"]
    assert len(rows) == 601 and rows[1][0] == "2019-09-06 12:00:00" and rows[-1][0] == "2019-09-06 12:09:59"
    v = np.array([[float(x) for x in row[1:]] for row in rows[1:]])
    assert ((v[:, 0] >= 0) & (v[:, 0] < 9000)).all()         # metersim.py:51
    assert (v[:, 1] >= 0).all() and (v[:, 1] > 0).any()       # tests/test_pvmodel.py:10; midday sun
    np.testing.assert_allclose(v[:, 2], v[:, 0] - v[:, 1], rtol=1e-12, atol=1e-9)   # pvsim.py:83
    d = np.load(npz)
    assert d["pv"].shape == (600, 8)
    np.testing.assert_array_equal(d["pv"][:, 0], v[:, 1])


@pytest.mark.gpu
def test_metersim_batch_messages(tmp_path):
    f = tmp_path / "m.jsonl"
    r = CliRunner().invoke(main, ["metersim", "--batch", "1", "--no-realtime", "--seconds", "30", "--out", str(f)])
    assert r.exit_code == 0, r.output
    msgs = [json.loads(line) for line in open(f)]
    assert len(msgs) == 30
    vals = np.array([json.loads(m["body"]) for m in msgs])
    assert ((vals >= 0) & (vals < 9000)).all()
    assert msgs[0]["timestamp"] == "2019-09-06T12:00:00"
