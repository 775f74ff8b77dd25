"""The MWT branch's workgroup cap as a function of the data-parallel world size
(network/dama.py _mwt_grid_cap): the measured world-1 cap at every world
size (RCCL's channels run on the CUs the cap leaves outside the MWT), and the override."""


def test_cap_world_size(monkeypatch):
    from network import dama
    monkeypatch.delenv('EWVIT_MWT_GRID_CAP', raising=False)
    assert dama._mwt_grid_cap(1) == dama.MWT_GRID_CAP == 128
    assert dama._mwt_grid_cap(2) == dama._mwt_grid_cap(8) == 128
    assert not hasattr(dama, 'RCCL_CU_RESERVE')
    monkeypatch.setenv('EWVIT_MWT_GRID_CAP', '96')
    assert dama._mwt_grid_cap(1) == dama._mwt_grid_cap(8) == 96
    monkeypatch.setenv('EWVIT_MWT_GRID_CAP', '0')
    assert dama._mwt_grid_cap(8) == 0                       # uncapped


def test_cap_without_process_group(monkeypatch):
    from network import dama
    monkeypatch.delenv('EWVIT_MWT_GRID_CAP', raising=False)
    assert dama._mwt_grid_cap() == dama.MWT_GRID_CAP          # no group: world 1
