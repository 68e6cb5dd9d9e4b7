"""Every drop-in name INTEGRATION.md §1 promises imports from where its table puts it
(the maintainer's path: `from tmhpvsim_amd import PVModel`, ...).  No GPU: only the
imports and the CPU-side objects are exercised."""
import importlib
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _table_rows():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    sec = text.split("## 1.")[1].split("## 2.")[0]
    rows = [l for l in sec.splitlines() if l.startswith("| `")]
    assert len(rows) >= 6
    out = []
    for r in rows:
        ref, drop = [c.strip() for c in r.strip("|").split("|")[:2]]
        ref_names = []
        for item in re.findall(r"`([^`]+)`", ref):
            if item.startswith(":") or ".py" in item:
                continue
            base = item.split("(")[0] if not item.endswith("(_file)") else item
            base = base.split(".")[-1]
            if base.endswith("(_file)"):
                ref_names += [base[:-len("(_file)")], base[:-len("(_file)")] + "_file"]
            else:
                ref_names.append(base.split("(")[0])
        targets = [t for t in re.findall(r"`([^`]+)`", drop) if t.startswith("tmhpvsim_amd")]
        out.append((ref_names, targets))
    return out


ROWS = _table_rows()


@pytest.mark.parametrize("ref_names,targets", ROWS, ids=[",".join(r[0]) for r in ROWS])
def test_integration_table_names_import(ref_names, targets):
    assert targets, "a drop-in row without a tmhpvsim_amd target"
    for t in targets:
        mod_name, _, attr = t.rpartition(".")
        try:   # a module target: it must hold every reference name of the row
            mod = importlib.import_module(t)
        except ModuleNotFoundError:
            mod = None
        if mod is not None:
            for n in ref_names:
                assert hasattr(mod, n), f"{t} lacks {n}"
            continue
        obj = getattr(importlib.import_module(mod_name), attr)   # an object target: `from mod import attr`
        assert attr in ref_names, f"{t} is not a name of the reference row {ref_names}"
        assert obj is not None


def test_top_level_from_imports():
    from tmhpvsim_amd import (BatchedSim, ClearskyindexModel, InterpolatedSampler, PVModel, Time,  # noqa: F401
                              get_meter_value)
    import tmhpvsim_amd
    assert tmhpvsim_amd.get_meter_value is importlib.import_module("tmhpvsim_amd.metersim").get_meter_value
    with pytest.raises(AttributeError):
        tmhpvsim_amd.no_such_name  # noqa: B018


def test_cpu_side_objects_behave_like_the_reference():
    import numpy as np
    from tmhpvsim_amd import InterpolatedSampler, Time, get_meter_value
    np.random.seed(3)
    v = get_meter_value()                 # metersim.py:49-51: 9000 U[0, 1)
    np.random.seed(3)
    assert v == 9000 * np.random.random() and 0.0 <= v < 9000.0
    t = Time(time=None, day_fraction=0.5, hour_fraction=0.25, min_fraction=0.0)   # clearskyindexmodel.py:42
    assert t.hour_fraction == 0.25
    s = InterpolatedSampler(lambda: 2.0)  # clearskyindexmodel.py:12-40: (before, after) then shift on next()
    before, after = s.before, s.after
    next(s)
    assert (s.before, s.after) == (after, 2.0)
    assert s.interpolate(0.25) == 0.25 * s.after + (1 - 0.25) * s.before
