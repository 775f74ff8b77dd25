"""TrainStep's capture preconditions for RCCL collectives (ewvit/graph.py _drain_watchdog,
verdict r4 item 6a): capturing with the process group's CUDA event cache on, or with no
flight-recorder status to drain the watchdog queue from, is a hard error (it brought back the
round-3 watchdog abort), unless EWVIT_ALLOW_UNDRAINED_CAPTURE=1.  The status probe itself
never raises: a torch build without the private dump reads as 'unavailable'."""
import types

import pytest

from ewvit import graph


class _Buckets:
    reduce = True


def _stub(monkeypatch, status):
    monkeypatch.setattr(graph.dist, 'get_backend', lambda group=None: 'nccl')
    monkeypatch.setattr(graph, '_pg_status', lambda: status)
    calls = []
    monkeypatch.setattr(graph, 'retire_eager_collectives', lambda: calls.append(1))
    st = types.SimpleNamespace(buckets=_Buckets(), group=None, _capture_mode='relaxed')
    return st, calls


def test_event_cache_on_refuses(monkeypatch):
    st, calls = _stub(monkeypatch, {'0': {'last_enqueued_collective': 1, 'last_completed_collective': 1}})
    monkeypatch.setenv('TORCH_NCCL_CUDA_EVENT_CACHE', '1')
    monkeypatch.delenv('EWVIT_ALLOW_UNDRAINED_CAPTURE', raising=False)
    with pytest.raises(RuntimeError, match='event cache'):
        graph.TrainStep._drain_watchdog(st)
    assert not calls


def test_no_flight_recorder_refuses(monkeypatch):
    st, calls = _stub(monkeypatch, {})
    monkeypatch.setenv('TORCH_NCCL_CUDA_EVENT_CACHE', '0')
    monkeypatch.delenv('EWVIT_ALLOW_UNDRAINED_CAPTURE', raising=False)
    with pytest.raises(RuntimeError, match='flight recorder'):
        graph.TrainStep._drain_watchdog(st)
    assert not calls


def test_preconditions_met_drains(monkeypatch):
    st, calls = _stub(monkeypatch, {'0': {'last_enqueued_collective': 3, 'last_completed_collective': 3}})
    monkeypatch.setenv('TORCH_NCCL_CUDA_EVENT_CACHE', '0')
    graph.TrainStep._drain_watchdog(st)
    assert calls == [1]


def test_override_warns(monkeypatch):
    st, calls = _stub(monkeypatch, {})
    monkeypatch.setenv('TORCH_NCCL_CUDA_EVENT_CACHE', '1')
    monkeypatch.setenv('EWVIT_ALLOW_UNDRAINED_CAPTURE', '1')
    with pytest.warns(UserWarning):
        graph.TrainStep._drain_watchdog(st)
    assert not calls


def test_status_probe_never_raises(monkeypatch):
    import torch._C._distributed_c10d as c10d
    monkeypatch.setattr(c10d, '_dump_nccl_trace_json', lambda **kw: (_ for _ in ()).throw(TypeError('no')),
                        raising=False)
    assert graph._pg_status() == {}
    monkeypatch.setattr(c10d, '_dump_nccl_trace_json', lambda **kw: 'not json', raising=False)
    assert graph._pg_status() == {}


def test_adam_load_state_after_release():
    """ewvit.optim.Adam refuses a state without entries for parameters a captured step
    updates; once TrainStep.close released the graphs (release_capture), it loads."""
    import torch
    from ewvit.optim import Adam
    w = torch.nn.Parameter(torch.randn(4))
    opt = Adam([w], lr=0.1)
    empty = opt.state_dict()                      # saved before any step: no per-parameter state
    opt.state[w] = {'step': torch.zeros(()), 'exp_avg': torch.zeros(4), 'exp_avg_sq': torch.zeros(4)}
    opt._captured_params = [w]                    # as finish_capture leaves it
    with pytest.raises(RuntimeError, match='captured step'):
        opt.load_state_dict(empty)
    opt.release_capture()
    opt.load_state_dict(empty)
    assert not opt.state
