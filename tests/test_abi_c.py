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


JNI_HARNESS = ROOT / "tests" / "c" / "jni_harness"


def test_jni_glue_built_and_exports_every_native(built):
    """libakka_gpu_jni.so (jvm/.../src/main/c/agx_jni.c) exports one Java_akka_dispatch_gpu_AgxJni_*
    symbol per `native` method of AgxJni.java."""
    import ctypes
    import re
    java = (ROOT / "jvm" / "akka-dispatch-gpu" / "src" / "main" / "java" / "akka" / "dispatch" / "gpu" /
            "AgxJni.java").read_text()
    natives = re.findall(r"static native \S+ (\w+)\(", java)
    assert len(natives) >= 20
    lib = ctypes.CDLL(str(ROOT / "akka_amd" / "lib" / "libakka_gpu_jni.so"))
    missing = [n for n in natives if not hasattr(lib, f"Java_akka_dispatch_gpu_AgxJni_{n}")]
    assert not missing, missing
    assert JNI_HARNESS.exists()


@pytest.mark.gpu
def test_jni_harness_on_gpu(built):
    """The JDK 8/11 binding end to end (tests/c/jni_harness.c): ActorModelSpec counts, per-actor
    bounded mailboxes, sender() ! reply to a JVM probe through the outbox, exceptions for errors."""
    r = subprocess.run([str(JNI_HARNESS)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "jni_harness OK" in r.stdout
