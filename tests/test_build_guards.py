"""Build-time guards of the kernel library (p2p_llm_chat_go_amd/_build.py), on the CPU.

The wide mid-M GEMM (csrc/kernels/wide_gemm.hip) streams its k loop through inline-asm
loads and LDS reads: the compiler cannot see which registers are still in flight, so a
spilled one would be read before it lands.  The build compiles that unit with the
resource-usage remarks and refuses any kernel with scratch; this checks the parser and,
when hipcc is present, the real unit."""
import os
import shutil
import subprocess

import pytest

from p2p_llm_chat_go_amd import _build as B


def test_scratch_remarks_are_refused():
    ok = ("x.hip:1:1: remark: Function Name: _Z1kv [-Rpass-analysis=kernel-resource-usage]\n"
          "x.hip:1:1: remark:     ScratchSize [bytes/lane]: 0 [-Rpass-analysis=kernel-resource-usage]\n")
    B.check_no_scratch("x.hip", ok)
    bad = ok + ("x.hip:2:1: remark: Function Name: _Z2k2v [-Rpass-analysis=kernel-resource-usage]\n"
                "x.hip:2:1: remark:     ScratchSize [bytes/lane]: 16 [-Rpass-analysis=kernel-resource-usage]\n")
    with pytest.raises(RuntimeError, match=r"_Z2k2v \(16 B/lane\)"):
        B.check_no_scratch("x.hip", bad)


@pytest.mark.skipif(not os.path.exists(B.HIPCC) and shutil.which("hipcc") is None,
                    reason="hipcc not installed")
def test_wide_gemm_compiles_without_scratch(tmp_path):
    src = os.path.join(B.CSRC, "kernels", "wide_gemm.hip")
    assert os.path.basename(src) in B.NO_SCRATCH
    r = subprocess.run([B.HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17",
                        "-munsafe-fp-atomics", "-I", os.path.join(B.CSRC, "include"),
                        "-I", os.path.join(B.CSRC, "kernels"), "--offload-device-only",
                        "-Rpass-analysis=kernel-resource-usage", "-c", src,
                        "-o", str(tmp_path / "wide.o")],
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-3000:]
    assert "Function Name: _ZN4wide16wide_gemm_kernel" in r.stdout
    B.check_no_scratch(src, r.stdout)
