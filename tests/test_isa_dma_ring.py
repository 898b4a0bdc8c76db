"""The LDS-DMA ring's cross-tile wait (cn_gemm.hip kDma: vmcnt(63) for a tile's first chunks, safe
only while every epilogue issues >= 63 - 8 vector-memory operations per wave) checked on the ISA of
the built library (CPU: llvm-objdump of its gfx950 code object, tools/isa_check.py), and the check
itself shown to fail on an epilogue trimmed below the bound."""
import os
import re
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import isa_check  # noqa: E402

LIB = os.path.join(ROOT, "cope-nerf_amd", "copenerf", "libcopenerf.so")


@pytest.fixture(scope="module")
def isa_text():
    if not os.path.exists(LIB):
        pytest.fail("libcopenerf.so not built (python -c 'import __graft_entry__ as g; g.build()')")
    return isa_check.disassemble(LIB)


def test_every_dma_ring_epilogue_covers_the_wait(isa_text):
    rep = isa_check.dma_ring_report(isa_text)
    # the 256x256 bf16 tile with image A operands: STORE, SOFTPLUS, RELU, MUL, TANGENT, BWD_SOFTPLUS,
    # BWD_RELU, SOFTPLUS_HEAD (fp32 A) and MUL / TANGENT / BWD_SOFTPLUS / BWD_RELU (image A)
    assert len(rep) >= 12, [r["kernel"] for r in rep]
    bad = [r for r in rep if not r["ok"]]
    assert not bad, bad
    assert all(r["ring_wait"] == 8 and r["need"] == 55 for r in rep)


def _trim_one_epilogue(text, kernel, keep):
    """The disassembly with the first >= 55-op epilogue block of `kernel` cut to `keep` stores."""
    lines = text.split("\n")
    start = next(i for i, ln in enumerate(lines) if ln.strip().endswith(f"<{kernel}>:"))
    out, run, trimmed = [], [], False

    def flush():
        nonlocal trimmed
        stores = [j for j, ln in enumerate(run) if re.match(r"\s*buffer_store", ln)]
        if not trimmed and len(stores) >= 55:
            drop = set(stores[keep:])
            run[:] = [ln for j, ln in enumerate(run) if j not in drop]
            trimmed = True
        out.extend(run)
        run.clear()

    for i, ln in enumerate(lines):
        if i <= start:
            out.append(ln)
            continue
        t = ln.strip()
        if re.match(r"^[0-9a-f]+ <.+>:$", t) or t.startswith(("s_branch", "s_cbranch")):
            run.append(ln)
            flush()
            continue
        run.append(ln)
    flush()
    assert trimmed
    return "\n".join(out)


def test_check_fails_on_a_trimmed_epilogue(isa_text):
    rep = isa_check.dma_ring_report(isa_text)
    k = next(r["kernel"] for r in rep if r["min_epilogue_vmem"] == 64)  # an image-only plain epilogue
    bad = isa_check.dma_ring_report(_trim_one_epilogue(isa_text, k, keep=40))
    r = next(r for r in bad if r["kernel"] == k)
    assert not r["ok"] and r["min_epilogue_vmem"] == 40, r
