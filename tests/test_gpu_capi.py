"""GPU: a plain C99 program drives the engine through the C ABI alone
(tests/c/abi_consumer.c): the per-packet drop-in, a ragged batch in compute
and verify mode, and with two or more devices the round-robin split."""
import subprocess

import pytest

from test_capi import build_abi_consumer

pytestmark = pytest.mark.gpu


def test_c_program_drives_the_gpu(tmp_path):
    exe = build_abi_consumer(tmp_path)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, f"abi_consumer failed check {r.returncode}: {r.stdout}{r.stderr}"
    assert r.stdout.startswith("abi 5 ok: 4 packets, slot 4224"), r.stdout
    assert "ctx_create 0, gpu leg ok" in r.stdout, r.stdout
