"""CPU tier: the provider's HBM store when its loader cannot start (a failed loader setup must
decline every request instead of reading an empty slot table or leaving waiters unanswered).

Here no HIP device exists, so the loader's setup (hipSetDevice, pinned ring, SDMA signals) fails the
way it does on a node where the provider sees no GPU; on the GPU box the same path is forced with
UDA_FAULT_STORE_SETUP (tests/test_gpu_mof_store.py)."""
import os
import time

import pytest

import uda_amd


def test_store_declines_when_its_loader_cannot_start(tmp_path):
    n = uda_amd.native()
    if n.device_count() > 0:
        pytest.skip("a HIP device is visible: the loader would start (GPU tier covers the injected failure)")
    f = tmp_path / "file.out"
    f.write_bytes(os.urandom(1 << 20))
    store = n.MofStore(64 << 20, [0])
    t0 = time.time()
    ok, why, _, _, _ = store.acquire("job_1", str(f), "holder-a")
    assert not ok and why, why  # the queued request is answered (declined), not left waiting
    time.sleep(0.5)  # the loader thread has given up by now
    ok2, why2, _, _, _ = store.acquire("job_1", str(f), "holder-b")
    assert not ok2 and "unavailable" in why2, why2  # later requests are declined at once
    assert time.time() - t0 < 30
    st = store.stats()
    assert st["declined"] >= 2 and st["resident_bytes"] == 0
    del store  # joins the (already finished) loader and its opener
