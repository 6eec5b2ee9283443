"""The lagged schedule's exchange form per rank (distributed.side_stream_wanted): beside the next gradient
kernel on a side stream only while one generation of workgroups covers the rank's launch, serialised on the
engine stream past it; DOPT_LAGGED_SIDE=1 / 0 force either form.  Host logic only (the CU count is given)."""
import pytest

import distributed as D


@pytest.mark.parametrize("n_local,want", [(1, True), (512, True), (513, False), (1024, False), (4096, False)])
def test_auto_follows_one_generation(monkeypatch, n_local, want):
    monkeypatch.delenv("DOPT_LAGGED_SIDE", raising=False)
    assert D.side_stream_wanted(n_local, cus=256) is want  # MI355X: 256 CUs x 2 resident workgroups


@pytest.mark.parametrize("knob,want", [("1", True), ("0", False)])
def test_knob_forces_the_form(monkeypatch, knob, want):
    monkeypatch.setenv("DOPT_LAGGED_SIDE", knob)
    for n_local in (64, 512, 4096):
        assert D.side_stream_wanted(n_local, cus=256) is want


def test_auto_spelled_out(monkeypatch):
    monkeypatch.setenv("DOPT_LAGGED_SIDE", "auto")
    assert D.side_stream_wanted(512, cus=256) and not D.side_stream_wanted(600, cus=256)
    assert D.side_stream_wanted(600, cus=304)  # more CUs, one generation again
