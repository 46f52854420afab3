#!/usr/bin/env python3
"""Member-kernel outputs vs the CPU member list for chosen C3 pairs (A/B build).

usage: DG_LIB_VARIANT=ab DG_MEMBERS=1 python scripts/member_debug.py 4242 4836 0
Prints per pair: members found on the device vs on the host, unverified members
(start, x, T, next start), and chunks whose verified prefix is short.
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CH, SLOTS = 2048, 2048 // 16 + 1


def host_members(R, V):
    r = np.frombuffer(R, np.uint8)
    v = np.frombuffer(V, np.uint8)
    E = min(len(r), len(v))
    mm = np.nonzero(r[:E] != v[:E])[0]
    pos = np.concatenate([[-1], mm, [E]])
    brk = np.nonzero(np.diff(pos) > 16)[0]
    starts = np.concatenate([[0], pos[brk + 1]])
    xs = pos[brk] + 1
    return starts, xs


def main():
    full = "--full" in sys.argv
    idx = [int(a) for a in sys.argv[1:] if a != "--full"] or [0]
    import torch
    from bench import CONFIGS, load_product
    from oracle.oracle import Oracle
    dg = load_product()
    L_ = dg.lib
    L_.dg_encode_plan_member_debug.argtypes = [C.c_void_p] + [C.POINTER(C.c_void_p)] * 4 + [C.POINTER(C.c_uint32)]
    hip = C.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    npg, L, rate, q, seed = CONFIGS["c3"][:5]
    ne = int(rate * L + 0.5)
    orc = Oracle()
    pairs = [orc.synth_pair(seed + i, L, ne) for i in idx]
    ctx = dg.Context(0)
    if full:   # the bench's whole batch, synthesised on the device
        n = npg
        ref = torch.empty(n * L, dtype=torch.uint8, device="cuda")
        ver = torch.empty(n * L, dtype=torch.uint8, device="cuda")
        ctx.check(L_.dg_synth_edit_pairs_device(ctx.handle, ref.data_ptr(), ver.data_ptr(), n, L, seed, ne,
                                                None), "synth")
    else:
        n = len(pairs)
        ref = torch.frombuffer(bytearray(b"".join(p[0] for p in pairs)), dtype=torch.uint8).cuda()
        ver = torch.frombuffer(bytearray(b"".join(p[1] for p in pairs)), dtype=torch.uint8).cuda()
    plan = dg.EncodePlan(ctx, "onepass", [(i * L, L, i * L, L) for i in range(n)], q=q)
    out = torch.empty(plan.output_bound, dtype=torch.uint8, device="cuda")
    offs = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    st = torch.empty(n, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    plan.run(ref.data_ptr(), ver.data_ptr(), out.data_ptr(), out.numel(), offs.data_ptr(), st.data_ptr())
    torch.cuda.synchronize()
    ptrs = [C.c_void_p() for _ in range(4)]
    nch = C.c_uint32()
    assert L_.dg_encode_plan_member_debug(plan.handle, *[C.byref(p) for p in ptrs], C.byref(nch)) == 0
    nc = nch.value
    mem_s = np.zeros(nc * SLOTS, np.uint32)
    srec = np.zeros((nc * SLOTS, 4), np.uint32)
    nmem = np.zeros(nc, np.uint32)
    csum = np.zeros((nc, 2), np.uint32)
    for a, p in zip([mem_s, srec, nmem, csum], ptrs):
        assert hip.hipMemcpy(a.ctypes.data, p, a.nbytes, 2) == 0
    per = nc // n
    okv = srec[:, 3].reshape(nc, SLOTS)
    cnts = nmem.astype(np.int64)
    unv = np.array([int((okv[g, :cnts[g]] == 0).sum()) for g in range(nc)]).reshape(n, per)
    print("unverified per pair: mean", unv.sum(1).mean(), "max", unv.sum(1).max(),
          "pairs with >2:", int((unv.sum(1) > 2).sum()), "worst", np.argsort(-unv.sum(1))[:6].tolist())
    for k, i in enumerate(idx):
        if full:
            k = i
        R, V = pairs[k]
        hs, hx = host_members(R, V)
        ds, dx, dok, dT = [], [], [], []
        short = []
        for c in range(per):
            g = k * per + c
            cnt = int(nmem[g])
            for j in range(cnt):
                ds.append(int(mem_s[g * SLOTS + j]))
                dx.append(int(srec[g * SLOTS + j, 0]))
                dok.append(int(srec[g * SLOTS + j, 3]))
            if csum[g, 0] != cnt:
                short.append((c, int(csum[g, 0]), cnt))
        ds = np.array(ds)
        same = len(ds) == len(hs) and bool((ds == hs).all())
        bad = [j for j in range(len(ds) - 1) if dok[j] == 0]
        print(f"pair {i}: status {int(st[k])} device members {len(ds)} host {len(hs)} starts_equal {same} "
              f"unverified {len(bad)} short_chunks {len(short)}")
        for j in bad[:12]:
            xh = hx[j] if j < len(hx) else -1
            print(f"   member {j}: s {ds[j]} x_dev {dx[j]} x_host {xh} T {xh - ds[j]} next {ds[j + 1]} "
                  f"chunk {ds[j] // CH} ok {dok[j]}")
        print("   short chunks (chunk, prefix, members):", short[:12])
    plan.close()


if __name__ == "__main__":
    main()
