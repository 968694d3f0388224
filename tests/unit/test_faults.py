import pytest

from multidisttorch_amd.runtime import faults


def test_parse_and_inject(monkeypatch):
    monkeypatch.setenv("MDT_FAULT", "trial=2,epoch=3")
    assert faults.parse_fault() == {"trial": 2, "epoch": 3}
    faults.maybe_inject(trial=2, epoch=2)
    with pytest.raises(faults.InjectedFault):
        faults.maybe_inject(trial=2, epoch=3, rank=0)
    monkeypatch.setenv("MDT_FAULT", "")
    faults.maybe_inject(trial=2, epoch=3)


def test_guarded_swallows_and_reports(capsys):
    seen = []
    with faults.guarded("t0", None, seen.append):
        raise ValueError("boom")
    assert isinstance(seen[0], ValueError)
    assert "t0 FAILED: ValueError: boom" in capsys.readouterr().out
