"""The plain-C driver of the ABI sequence the JVM shim uses (tests/c/abi_sequence.c,
built by __graft_entry__.build()): ActorModelSpec received == processed from 200 sender
threads, MailboxConfigSpec bounded overflow, error codes, stats without read-back."""
import pathlib
import subprocess

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
BIN = ROOT / "tests" / "c" / "abi_sequence"


def test_abi_sequence_binary_built(built):
    assert BIN.exists(), "build() compiles tests/c/abi_sequence.c"


@pytest.mark.gpu
def test_abi_sequence_on_gpu(built):
    r = subprocess.run([str(BIN)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "abi_sequence OK" in r.stdout
