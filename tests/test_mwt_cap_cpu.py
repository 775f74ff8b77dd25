"""The MWT branch's workgroup cap as a function of the data-parallel world size
(network/dama.py _mwt_grid_cap): the measured world-1 cap, RCCL's CU
reserve taken off the MWT's half of the chip at world > 1, and the environment overrides."""
import pytest


def test_cap_world_size(monkeypatch):
    from network import dama
    monkeypatch.delenv('EWVIT_MWT_GRID_CAP', raising=False)
    monkeypatch.delenv('EWVIT_RCCL_CU_RESERVE', raising=False)
    assert dama._mwt_grid_cap(1) == dama.MWT_GRID_CAP == 96
    # the default reserve leaves the MWT's 128-CU share above the world-1 cap
    assert dama._mwt_grid_cap(8) == min(dama.MWT_GRID_CAP, dama.MWT_CU_SHARE - dama.RCCL_CU_RESERVE) == 96
    monkeypatch.setenv('EWVIT_RCCL_CU_RESERVE', '48')
    assert dama._mwt_grid_cap(2) == 128 - 48
    monkeypatch.setenv('EWVIT_RCCL_CU_RESERVE', '1000')
    assert dama._mwt_grid_cap(2) == 64                      # never below 64 workgroups
    monkeypatch.setenv('EWVIT_MWT_GRID_CAP', '128')
    assert dama._mwt_grid_cap(1) == dama._mwt_grid_cap(8) == 128


def test_cap_without_process_group(monkeypatch):
    from network import dama
    monkeypatch.delenv('EWVIT_MWT_GRID_CAP', raising=False)
    assert dama._mwt_grid_cap() == dama.MWT_GRID_CAP          # no group: world 1
