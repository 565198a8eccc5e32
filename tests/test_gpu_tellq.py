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


def test_tell_burst_beyond_capacity_is_delivered(built):
    """A burst of agx_tell 10x the engine's msg_capacity, from 4 threads, to an idle engine: nothing
    refused or lost (an unbounded mailbox never refuses an enqueue, AbstractNodeQueue.java:79-82).
    Each pump takes what fits beside the mail in flight; agx_pump_idle reschedules while tells wait.
    After every pump: staged + emitted = delivered + dead + in flight, in flight <= msg_capacity."""
    n = 1024
    cap = 4 * n
    eng = GpuEngine(EngineConfig(n_actors=n, throughput=5, capacity=0, n_words=2, max_emit=1, msg_capacity=cap))
    eng.register_range(0, n, Kind.COUNTER)
    threads, per = 4, 10 * cap // 4
    rng = np.random.default_rng(11)
    dsts = [rng.integers(0, 64, per).astype(np.uint32) for _ in range(threads)]  # (64 hot actors: deep queues)
    subs = [0]
    lock = threading.Lock()

    def sender(t):
        k = 0
        for d in dsts[t].tolist():
            k += eng.tell_one(d, 1 + (d & 7), NO_SENDER)
        with lock:
            subs[0] += k

    ths = [threading.Thread(target=sender, args=(t,)) for t in range(threads)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert subs[0] == 1  # one submission for the whole burst
    pumps, again = 0, True
    while again:
        pumps += 1
        assert pumps < 10_000
        st = eng.run()
        assert st.staged + st.emitted == st.delivered + st.dead_letters + st.in_flight
        assert st.in_flight <= cap
        again = eng.pump_idle()
    st = eng.stats()
    assert pumps >= 10  # (10x the capacity: at least 10 pumps)
    assert st.staged == threads * per and st.delivered == threads * per and st.dead_letters == 0
    assert st.in_flight == 0
    w = eng.read_state()[0].T  # (actor-major rows -> word-major)
    allp = np.concatenate(dsts)
    cnt = np.bincount(allp, minlength=n)
    assert np.array_equal(w[0], cnt.astype(np.uint64))
    assert np.array_equal(w[1], (cnt * (1 + (np.arange(n) & 7))).astype(np.uint64))
    eng.close()


def test_stage_tells_all_or_nothing(built):
    """agx_stage_tells beyond capacity: AGX_ECAPACITY with nothing staged and no counter moved; a
    tagged sender (AGX_EINVAL) likewise; a burst that fits is then accepted and delivered."""
    from akka_amd._lib import AgxError
    n = 512
    eng = GpuEngine(EngineConfig(n_actors=n, throughput=5, capacity=0, n_words=2, max_emit=1, msg_capacity=4 * n))
    eng.register_range(0, n, Kind.COUNTER)
    eng.tell(np.arange(n, dtype=np.uint32), 1)
    eng.run(1)  # (throughput 5: all n delivered in one superstep; nothing in flight)
    eng.tell(np.zeros(3 * n, np.uint32), 1)  # 3n in flight after a run of 0 supersteps
    before = eng.stats()
    with pytest.raises(AgxError) as ei:
        eng.tell(np.arange(2 * n, dtype=np.uint32) % n, 1)  # 3n + 2n > 4n
    assert "nothing staged" in str(ei.value)
    after = eng.stats()
    assert after == before
    with pytest.raises(AgxError):
        eng.tell(np.array([1, 2], np.uint32), 1, src=np.array([5, 0x80000001], np.uint32))
    assert eng.stats() == before
    eng.tell(np.arange(n, dtype=np.uint32), 1)  # 3n + n = 4n: fits
    st = eng.run()
    assert st.staged == 5 * n and st.delivered == 5 * n and st.in_flight == 0
    assert st.staged + st.emitted == st.delivered + st.dead_letters + st.in_flight
    eng.close()


def test_pump_budget_reschedules_and_cancel(built):
    """A pump that stops at its superstep budget with mail in flight asks to run again (Mailbox.run
    re-registers while hasMessages, Mailbox.scala:227-240), and keeps the engine scheduled meanwhile;
    agx_pump_cancel returns it to idle (Dispatcher.scala:130-138)."""
    eng = GpuEngine(EngineConfig(n_actors=2048, throughput=5, capacity=0, n_words=2, max_emit=1))
    eng.register_range(0, 2048, Kind.COUNTER)
    assert sum(eng.tell_one(7, i) for i in range(1, 101)) == 1
    pumps, again = 0, True
    while again:
        pumps += 1
        eng.run(1, stats=False)
        again = eng.pump_idle()
        if again and pumps == 1:
            assert not eng.tell_one(8, 1)  # still scheduled: no second pump
    assert pumps == 20
    w = eng.read_state()[0].T  # (actor-major rows -> word-major)
    assert w[0][7] == 100 and w[1][7] == 5050 and w[0][8] == 1
    assert eng.tell_one(9, 1)
    eng.pump_cancel()
    assert eng.tell_one(9, 2)  # idle again after the cancel: this tell submits
    eng.run()
    assert not eng.pump_idle()
    assert eng.read_state()[0][9][0] == 2
    eng.close()
