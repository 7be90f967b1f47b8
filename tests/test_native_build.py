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


ASAN_PROBE = r'''
import sys, torch
torch.ops.load_library(sys.argv[1])
o = torch.ops.ina
assert o.abi_version() >= 6 and o.rec_attn_ok(20, 37) and not o.rec_attn_ok(24, 37)
cpu = torch.zeros(8)
calls = [
    lambda: o.slab_reduce(torch.zeros(3), torch.zeros(2), False),
    lambda: o.adam_step(cpu, cpu, cpu, cpu, None, 1e-3, 1, .9, .999, 1e-8, 1., 0., None, None, None, None),
    lambda: o.adagrad_step(cpu, cpu, cpu, None, 1e-3, 1., 0., None, None, None),
    lambda: o.nonfinite_flag(cpu, None, cpu),
    lambda: o.sample_episodes(torch.zeros(4, 2, dtype=torch.int32), 2, 2, 1, 1, 0, 0.0, None, None),
    lambda: o.routing_fwd(torch.zeros(10, 40), torch.zeros(40, 40), 1, 5, 1, 1, 3, 0),
]
raised = 0
for f in calls:
    try:
        f()
    except Exception:
        raised += 1
print("raised", raised, "of", len(calls))
assert raised == len(calls)
'''


@pytest.mark.slow
def test_host_bindings_under_asan(tmp_path):
    """the host code (torch op bindings + launch stubs) built with -fsanitize=address
    (host only; GPU code is not instrumented) loads and runs its argument-validation paths clean in a
    CPU process (gcc's libasan + libstdc++ preloaded; leak checks off -- the interpreter never frees
    everything)."""
    env = dict(os.environ, INA_ASAN="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "csrc", "build.py")], env=env, capture_output=True,
                       text=True, timeout=1500)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lib = r.stdout.strip().splitlines()[-1]
    assert lib.endswith("_ina_kernels_asan.so") and os.path.exists(lib)
    gcc = lambda n: subprocess.run(["gcc", f"-print-file-name={n}"], capture_output=True, text=True).stdout.strip()
    probe = tmp_path / "probe.py"
    probe.write_text(ASAN_PROBE)
    env = dict(os.environ, LD_PRELOAD=f"{gcc('libasan.so')} {gcc('libstdc++.so.6')}",
               ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=0")
    env.pop("INA_ASAN", None)
    out = subprocess.run([sys.executable, str(probe), lib], env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0 and "ERROR: AddressSanitizer" not in out.stderr, out.stdout + out.stderr[-4000:]
    assert "raised 6 of 6" in out.stdout
