"""The MWT branch's workgroup cap as a function of the data-parallel world size
(network/dama.py _mwt_grid_cap): the measured world-1 cap, RCCL's CU
reserve taken off it at world > 1, and the environment overrides."""
import pytest


def test_cap_world_size(monkeypatch):
    from network import dama
    monkeypatch.delenv('EWVIT_MWT_GRID_CAP', raising=False)
    monkeypatch.delenv('EWVIT_RCCL_CU_RESERVE', raising=False)
    assert dama._mwt_grid_cap(1) == dama.MWT_GRID_CAP == 128
    assert dama._mwt_grid_cap(8) == dama.MWT_GRID_CAP - dama.RCCL_CU_RESERVE
    monkeypatch.setenv('EWVIT_RCCL_CU_RESERVE', '32')
    assert dama._mwt_grid_cap(2) == dama.MWT_GRID_CAP - 32
    monkeypatch.setenv('EWVIT_RCCL_CU_RESERVE', '1000')
    assert dama._mwt_grid_cap(2) == 64                      # never below 64 workgroups
    monkeypatch.setenv('EWVIT_MWT_GRID_CAP', '96')
    assert dama._mwt_grid_cap(1) == dama._mwt_grid_cap(8) == 96


def test_cap_without_process_group(monkeypatch):
    from network import dama
    monkeypatch.delenv('EWVIT_MWT_GRID_CAP', raising=False)
    assert dama._mwt_grid_cap() == dama.MWT_GRID_CAP          # no group: world 1
