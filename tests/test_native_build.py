"""The gfx950 kernel library builds (cross-compiled, no GPU needed) and registers every op."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OPS = ["abi_version", "lstm_fwd", "lstm_bwd", "attn_fwd", "attn_bwd", "routing_fwd", "routing_bwd", "ntn_fwd",
       "ntn_bwd", "adam_step", "adagrad_step", "slab_reduce", "sample_episodes"]


def test_library_builds_and_registers_ops():
    sys.path.insert(0, os.path.join(ROOT, "csrc"))
    import build as b
    lib = b.build()
    assert os.path.exists(lib)
    code = ("import torch; torch.ops.load_library(%r); "
            "print(','.join(n for n in %r if hasattr(torch.ops.ina, n)))" % (lib, OPS))
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip().split(",") == OPS


def test_code_objects_target_gfx950():
    lib = os.path.join(ROOT, "induction_network_on_fewrel_amd", "_ina_kernels.so")
    if not os.path.exists(lib):
        pytest.skip("library not built")
    data = open(lib, "rb").read()
    assert b"gfx950" in data


def test_gpu_path_fails_loudly_without_kernels(monkeypatch):
    """A GPU run must never silently fall back: ops() raises when the library cannot load."""
    from induction_network_on_fewrel_amd.ops import _ext
    monkeypatch.setattr(_ext, "_loaded", False)
    monkeypatch.setattr(_ext, "_LIB", "/nonexistent/_ina_kernels.so")
    with pytest.raises(RuntimeError):
        _ext.ops()
