"""The lock-free tell path (akka_amd/csrc/agx_tellq.h: agx_tell / agx_pump_idle) on the CPU:
tests/c/tellq_test.cpp checks that a burst to an idle engine submits one pump (Mailbox.setAsScheduled,
Mailbox.scala:185-194), and that 8 producer threads racing a self-resubmitting pump lose no tell,
keep each producer's order and lose no wake-up -- plain, and under ThreadSanitizer (host code only)."""
import pathlib
import subprocess

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
SRC = ROOT / "tests" / "c" / "tellq_test.cpp"


@pytest.mark.parametrize("flags", [["-O2"], ["-O1", "-g", "-fsanitize=thread"]], ids=["plain", "tsan"])
def test_tell_queue(tmp_path, flags):
    exe = tmp_path / "tellq_test"
    subprocess.run(["g++", "-std=c++17", "-pthread", "-Wall", *flags, "-o", str(exe), str(SRC)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "one submission per burst OK" in r.stdout and "none lost OK" in r.stdout
    assert "bounded:" in r.stdout
    assert "WARNING: ThreadSanitizer" not in r.stderr, r.stderr[-3000:]
