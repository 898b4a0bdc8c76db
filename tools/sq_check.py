"""Tile A/B at the C2 layer shape: every bf16x6 epilogue on the default tiles vs the
256x256 tile (COPENERF_X6_SQ, read at library load, so each variant is a subprocess).
Prints per-epilogue µs and checks the outputs are bitwise equal (same MFMA chain order)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child():
    import torch
    sys.path[:0] = [os.path.join(ROOT, "cope-nerf_amd"), ROOT]
    from copenerf import ops
    M, N, K = int(os.environ.get("M", 524288)), 256, 256
    g = torch.Generator(device="cuda").manual_seed(0)
    A = torch.randn(M, K, device="cuda", generator=g) * 0.1
    B = torch.randn(N, K, device="cuda", generator=g) * 0.05
    bias = torch.randn(N, device="cuda", generator=g) * 0.1
    aux0 = torch.rand(M, N, device="cuda", generator=g) * 0.02
    aux1 = torch.randn(M, N, device="cuda", generator=g)
    aux2 = torch.randn(M, N, device="cuda", generator=g)
    Bs = ops.split_bf16x3(B)
    sg = dict(aux0=aux0, aux_beta=100.0)
    so = dict(sg, aux1=aux1, aux2=aux2, aux2_scale=100.0)
    out = {}
    for name, epi, kw in (("store", ops.EPI_STORE, dict(bias=bias)), ("softplus", ops.EPI_SOFTPLUS, dict(bias=bias)),
                          ("relu", ops.EPI_RELU, dict(bias=bias)), ("mul", ops.EPI_MUL, sg),
                          ("tangent", ops.EPI_TANGENT, sg), ("bwd_softplus", ops.EPI_BWD_SOFTPLUS, so),
                          ("bwd_relu", ops.EPI_BWD_RELU, dict(aux0=aux1)),
                          ("main", 7, {})):
        o0 = torch.zeros(M, N, device="cuda")
        fn = lambda: ops.linear(A, Bs, N, K, o0, epi, **kw)  # noqa: E731
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        out[name] = (us, o0.double().sum().item(), o0.view(torch.int32).long().sum().item())
    print("RESULT", repr(out), flush=True)


def main():
    if os.environ.get("SQ_CHILD"):
        return child()
    variants = sys.argv[1:] or ["0", "0x7e"]
    res = {}
    for rnd in range(2):
        for v in variants:
            env = dict(os.environ, SQ_CHILD="1", COPENERF_X6_SQ=v)
            r = subprocess.run([sys.executable, __file__], env=env, capture_output=True, text=True, timeout=300)
            line = [x for x in r.stdout.splitlines() if x.startswith("RESULT")]
            if r.returncode != 0 or not line:
                print(r.stdout[-2000:], r.stderr[-2000:])
                sys.exit(1)
            res.setdefault(v, []).append(eval(line[0][7:]))
            print(f"round {rnd} X6_SQ={v}: " + "  ".join(f"{k} {t[0]:.1f}" for k, t in res[v][-1].items()), flush=True)
    base = res[variants[0]][0]
    for v in variants[1:]:
        for k, t in res[v][0].items():
            if k != "main":
                print(f"X6_SQ={v} {k}: bitwise {'EQUAL' if t[2] == base[k][2] else 'DIFFERENT'} "
                      f"(sum {t[1]:.6e} vs {base[k][1]:.6e})")


if __name__ == "__main__":
    main()
