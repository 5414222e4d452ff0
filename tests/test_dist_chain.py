"""CPU: the N > 1 measurement decision of bench.py (`dist.run_chain`): which path is measured when the persistent
multi-GPU schedule applies, does not apply, or fails its self-check / timed-launch check, and that RCCL is the
fallback everywhere except on one GPU (where RCCL refuses two ranks per device). The GPU rehearsal of the same
chain with an injected publish failure is `tests/test_gpu_dist_persist.py::test_bench_two_ranks_drop_publish`."""
import pytest

import fem355  # noqa: F401
from fem355 import _capi as C, dist, dist_persist


def chain(path, same_gpu, persist_result, log=None):
    calls = []

    def persist():
        calls.append("persist")
        if isinstance(persist_result, Exception):
            raise persist_result
        return persist_result

    def rccl():
        calls.append("rccl")
        return {"value": 1.0, "path": "rccl"}

    out, used = dist.run_chain(path, same_gpu, persist, rccl, log=log or (lambda m: None))
    return out, used, calls


def test_persist_ok_is_measured():
    out, used, calls = chain("auto", False, (True, {"value": 2.0}))
    assert used == "persist" and out == {"value": 2.0} and calls == ["persist"]


@pytest.mark.parametrize("result", [(False, None), C.FemError("capacity")])
def test_failed_or_unavailable_persist_falls_back_to_rccl(result):
    msgs = []
    out, used, calls = chain("auto", False, result, log=msgs.append)
    assert used == "rccl" and calls == ["persist", "rccl"] and out["path"] == "rccl"
    assert any("RCCL" in m for m in msgs)


@pytest.mark.parametrize("result", [(False, None), C.FemError("ipc")])
def test_same_gpu_or_forced_persist_raises(result):
    for path, same in (("auto", True), ("persist", False), ("persist", True)):
        with pytest.raises(RuntimeError, match="no RCCL fallback"):
            chain(path, same, result)


def test_rccl_only_path_never_tries_persist():
    out, used, calls = chain("rccl", False, (True, {"value": 2.0}))
    assert used == "rccl" and calls == ["rccl"]


def test_attempt_order_is_fine_grained_first():
    # fine-grained comm blocks (coherent for peer GPUs by construction) until a real multi-GPU run
    # has shown hipMalloc memory coherent across GPUs
    assert dist_persist.ATTEMPTS == ("fine-grained", "coarse-grained")
