"""The lock-free tell path against the engine on the GPU (agx_tell from several host threads while
one pump thread runs agx_run + agx_pump_idle): every tell delivered exactly once, a pump submitted
only on idle -> scheduled, and the final state equal to the oracle's for the same tells (COUNTER
actors: count and sum do not depend on how the senders interleave).  ctypes releases the GIL
during each foreign call, so the tells really race the pump.  Reference: AbstractNodeQueue.java:79-82,
Mailbox.scala:185-194, ActorModelSpec.scala:323-336."""
import threading

import numpy as np
import pytest

from akka_amd.engine import EngineConfig, GpuEngine, Kind, NO_SENDER

pytestmark = pytest.mark.gpu


def test_tell_from_threads_with_pump(built):
    from oracle import BspOracle
    n, threads, per = 50_000, 4, 20_000
    cfg = dict(n_actors=n, throughput=5, capacity=0, n_words=2, max_emit=1)
    eng = GpuEngine(EngineConfig(**cfg))
    eng.register_range(0, n, Kind.COUNTER)
    rng = np.random.default_rng(3)
    dsts = [rng.integers(0, n + 10, per).astype(np.uint32) for _ in range(threads)]  # (10 unknown refs)
    pays = [rng.integers(0, 1000, per).astype(np.uint32) for _ in range(threads)]
    submitted = [0]
    lock = threading.Lock()
    done = threading.Event()

    def sender(t):
        for d, p in zip(dsts[t].tolist(), pays[t].tolist()):
            if eng.tell_one(d, p, NO_SENDER):
                with lock:
                    submitted[0] += 1

    def pump():
        ran = 0
        while True:
            with lock:
                pending = submitted[0] > ran
            if not pending:
                if done.is_set():
                    with lock:
                        if submitted[0] == ran:
                            return ran
                continue
            ran += 1
            eng.run()
            if eng.pump_idle():
                with lock:
                    submitted[0] += 1

    ths = [threading.Thread(target=sender, args=(t,)) for t in range(threads)]
    runs = []
    pt = threading.Thread(target=lambda: runs.append(pump()))
    pt.start()
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    done.set()
    pt.join(timeout=120)
    assert not pt.is_alive(), "the pump never drained the tells (lost wake-up)"
    sg = eng.stats()
    assert sg.staged == threads * per and sg.in_flight == 0
    assert 1 <= runs[0] <= threads * per
    assert not eng.pump_idle()  # (idle: nothing published since)
    ref = BspOracle(**cfg)
    ref.register_range(0, n, Kind.COUNTER)
    ref.tell(np.concatenate(dsts), np.concatenate(pays))
    so = ref.run()
    for k in ("delivered", "dead_letters", "unhandled", "emitted", "staged", "in_flight"):
        assert getattr(sg, k) == so[k], (k, getattr(sg, k), so[k])
    assert np.array_equal(eng.read_state()[0], ref.read_state()[0])
    eng.close()


def test_tell_burst_one_submission(built):
    eng = GpuEngine(EngineConfig(n_actors=4096, throughput=5, capacity=0, n_words=2, max_emit=1))
    eng.register_range(0, 4096, Kind.COUNTER)
    subs = sum(eng.tell_one(i % 4096, 1) for i in range(10_000))
    assert subs == 1
    st = eng.run()
    assert st.delivered == 10_000 and not eng.pump_idle()
    assert eng.tell_one(5, 1)  # idle again: the next tell submits
    eng.close()
