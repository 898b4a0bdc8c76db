"""Static checks on the gfx950 ISA of the built libcopenerf.so (CPU only: llvm-objdump).

The LDS-DMA ring of the 256x256 bf16 linear tile (cn_gemm.hip, `kDma` in linear_kernel) waits for
the first DNS - 1 chunks of every tile after the first with `s_waitcnt vmcnt(63)`: those chunks'
pieces were issued before the previous tile's epilogue, vmcnt retires loads, stores and LDS-DMA in
issue order, and 63 is the counter's largest wait.  That is safe only if, between the pieces and the
wait, at least 63 - W younger vector-memory operations are issued, W the ring's own wait
(`vmcnt(4 * (DNS - 2))`: the DNS - 2 later chunks' pieces) -- i.e. every epilogue issues at least
63 - W of them.  The one exception is SOFTPLUS_HEAD with no stored output (the sampler's sdf-only
launch, `epi_big` false), which takes the ring's own wait instead.

    python tools/isa_check.py [path/to/libcopenerf.so]

dma_ring_report() walks each kDma kernel's control-flow graph.  The epilogue region is every block
reachable from an exit of the chunk loop (the smallest natural loop holding the MFMAs) before the
vmcnt(63) wait.  The direct epilogues are fully unrolled and branch-free per element, so each output
variant is one basic block holding all of its memory operations: every region block that issues
vector-memory operations must issue at least 63 - W of them, unless every path from it to the wait
passes an `s_waitcnt vmcnt(0)` (everything older retired: SOFTPLUS_HEAD's epilogue, whose row sums
cross a barrier), or every path from the chunk loop to it does (the ring's pieces retired before the
block issues anything: the head epilogues' row stores after that barrier).  The dispatch between the variants cannot skip all of them (the host requires out0
or out0_b), which the graph alone does not show.  `flat_*` instructions in the region (which vmcnt
does not order) fail the check too."""
from __future__ import annotations

import heapq
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/llvm/bin"
_ADDR = re.compile(r"^([0-9a-f]+) <(.+)>:$")
_BR = re.compile(r"^s_(c?branch\w*)\s+(L\d+)")
EPI_SOFTPLUS_HEAD = 8


def disassemble(so_path: str) -> str:
    """llvm-objdump of the gfx950 code object inside the library's offload bundle."""
    with tempfile.TemporaryDirectory() as d:
        fat, co = os.path.join(d, "fatbin.bin"), os.path.join(d, "co.o")
        subprocess.run([f"{LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={fat}", so_path, os.path.join(d, "x")],
                       check=True, capture_output=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fat}", f"--output={co}"],
                       check=True, capture_output=True)
        return subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--symbolize-operands", co], check=True,
                              capture_output=True, text=True).stdout


def parse_kernels(text: str) -> dict:
    """{kernel symbol: [block, ...]}, block = {"label", "ins": [mnemonic + operands], "succ": [index]}.
    Blocks start at branch-target labels and after every branch."""
    kernels, cur = {}, None
    for line in text.split("\n"):
        m = _ADDR.match(line.strip())
        if m:
            name = m.group(2)
            if re.fullmatch(r"L\d+", name):
                if cur is not None:
                    cur.append({"label": name, "ins": []})
            else:
                cur = [{"label": None, "ins": []}]
                kernels[name] = cur
            continue
        if cur is None:
            continue
        t = line.strip().split("//")[0].strip()
        if not t or t.startswith(("Disassembly", ".")):
            continue
        cur[-1]["ins"].append(t)
        if t.startswith(("s_branch", "s_cbranch", "s_endpgm", "s_setpc", "s_trap")):
            cur.append({"label": None, "ins": []})
    for name, blocks in kernels.items():
        blocks[:] = [b for b in blocks if b["ins"] or b["label"]]
        index = {b["label"]: i for i, b in enumerate(blocks) if b["label"]}
        for i, b in enumerate(blocks):
            last = b["ins"][-1] if b["ins"] else ""
            succ = []
            m = _BR.match(last)
            if m:
                succ.append(index[m.group(2)])
                if m.group(1) != "branch" and i + 1 < len(blocks):
                    succ.append(i + 1)
            elif not last.startswith(("s_endpgm", "s_setpc", "s_trap")) and i + 1 < len(blocks):
                succ.append(i + 1)
            b["succ"] = succ
    return kernels


def _vmem(ins: str) -> bool:
    return ins.startswith(("buffer_", "global_", "scratch_", "flat_"))


def _epilogue_of(symbol: str) -> int | None:
    """The EPI template argument of a cn::linear_kernel symbol (its 8th)."""
    m = re.match(r"_ZN2cn13linear_kernelI((?:L[ib]\d+E)+)E", symbol)
    if not m:
        return None
    args = re.findall(r"L[ib](\d+)E", m.group(1))
    return int(args[7]) if len(args) > 7 else None


def _dominators(blocks) -> list:
    """dom[k] = the set of blocks dominating k (entry 0), iteratively."""
    n = len(blocks)
    preds = [[] for _ in range(n)]
    for k, b in enumerate(blocks):
        for s in b["succ"]:
            preds[s].append(k)
    full = set(range(n))
    dom = [full] * n
    dom[0] = {0}
    changed = True
    while changed:
        changed = False
        for k in range(1, n):
            ps = [dom[p] for p in preds[k]]
            d = (set.intersection(*ps) if ps else set()) | {k}
            if d != dom[k]:
                dom[k], changed = d, True
    return dom, preds


def _ring_loop(blocks, mfma) -> set:
    """The chunk loop: the smallest natural loop (back edge b -> h, h dominating b: h plus every
    block reaching b without passing h) that contains an MFMA block.  The tile loop contains it."""
    dom, preds = _dominators(blocks)
    best = None
    for b, blk in enumerate(blocks):
        for h in blk["succ"]:
            if h not in dom[b]:
                continue
            body, stack = {h}, [b]
            while stack:
                k = stack.pop()
                if k in body:
                    continue
                body.add(k)
                stack.extend(preds[k])
            if body & mfma and (best is None or len(body) < len(best)):
                best = body
    return best or set()


def dma_ring_report(text: str) -> list:
    """One entry per kernel with an LDS-DMA ring wait (vmcnt(63) beside `buffer_load ... lds`):
    {"kernel", "ring_wait" (W), "need" (63 - W), "min_epilogue_vmem", "flat_on_path", "ok"}."""
    out = []
    for name, blocks in parse_kernels(text).items():
        ins_all = [i for b in blocks for i in b["ins"]]
        if not any(i.startswith("buffer_load") and i.endswith(" lds") for i in ins_all):
            continue
        w63 = [k for k, b in enumerate(blocks) if any(i.startswith("s_waitcnt vmcnt(63)") for i in b["ins"])]
        if not w63:
            continue
        # the ring's own wait: the vmcnt(N) the wait-select blocks after vmcnt(63) hold
        ring = None
        for k in range(max(0, w63[0] - 4), min(w63[0] + 4, len(blocks))):
            for i in blocks[k]["ins"]:
                m = re.fullmatch(r"s_waitcnt vmcnt\((\d+)\)", i)
                if m and int(m.group(1)) != 63:
                    ring = int(m.group(1))
        mfma = {k for k, b in enumerate(blocks) if any(i.startswith("v_mfma") for i in b["ins"])}
        loop = _ring_loop(blocks, mfma)
        # the epilogue starts where the chunk loop exits
        starts = {s for k in loop for s in blocks[k]["succ"] if s not in loop}
        drains = {k for k, b in enumerate(blocks) if any(re.match(r"s_waitcnt vmcnt\(0\)", i) for i in b["ins"])}
        # the epilogue region: blocks reachable from the loop's exits before the ring's wait
        region, stack = set(), list(starts)
        while stack:
            k = stack.pop()
            if k in region or k in loop or k in w63:
                continue
            region.add(k)
            stack.extend(blocks[k]["succ"])

        def undrained_to_wait(k):
            """W63 reachable from the end of block k without an s_waitcnt vmcnt(0) on the way."""
            seen, st = set(), list(blocks[k]["succ"])
            while st:
                j = st.pop()
                if j in seen or j in drains or j in mfma:
                    continue
                if j in w63:
                    return True
                seen.add(j)
                st.extend(blocks[j]["succ"])
            return False

        # blocks reachable from the loop's exits without passing a drain
        undrained, stack = set(), [s for s in starts if s not in drains]
        while stack:
            k = stack.pop()
            if k in undrained or k in loop or k in w63 or k in drains:
                continue
            undrained.add(k)
            stack.extend(blocks[k]["succ"])

        # every block issuing vector-memory operations issues enough of them itself, or is preceded or followed
        # by a drain on every path to the wait (the direct epilogues are fully unrolled: one block
        # per output variant; the host requires out0 or out0_b, so no variant stores nothing)
        best, flat = None, False
        for k in region:
            nv = sum(1 for i in blocks[k]["ins"] if _vmem(i))
            flat = flat or any(i.startswith("flat_") for i in blocks[k]["ins"])
            if nv == 0 or k in drains or k not in undrained or not undrained_to_wait(k):
                continue
            best = nv if best is None else min(best, nv)
        need = 63 - (ring if ring is not None else 0)
        out.append({"kernel": name, "ring_wait": ring, "need": need, "min_epilogue_vmem": best,
                    "epilogue_blocks": len(region), "flat_on_path": flat,
                    "ok": ring is not None and bool(region) and (best is None or best >= need) and not flat})
    return out


def main():
    so = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                           "cope-nerf_amd", "copenerf", "libcopenerf.so")
    rep = dma_ring_report(disassemble(so))
    for r in rep:
        print(("ok  " if r["ok"] else "BAD ") + f"ring wait {r['ring_wait']}, epilogue >= {r['min_epilogue_vmem']} "
              f"vmem ops (need {r['need']})  {r['kernel']}")
    sys.exit(0 if rep and all(r["ok"] for r in rep) else 1)


if __name__ == "__main__":
    main()
