import sys, random
sys.path.insert(0, 'tests'); sys.path.insert(0, 'oracle')
from conftest import load_product
import oracle as O
dg = load_product(); o = O.Oracle(); ctx = dg.Context(0)
import torch
bad = []
for n in list(range(300, 420)) + [737, 1537, 3700, 10340]:
    d = random.Random(n).randbytes(n)
    if dg.crc64_xz(d, ctx=ctx) != o.crc64_xz(d): bad.append(n)
print("host-api bad lengths:", bad[:40], len(bad))
# same via batch on a larger buffer (like decode's output buffer)
for n in [340, 737, 3700]:
    d = random.Random(n).randbytes(n)
    t = torch.zeros(n + 4096, dtype=torch.uint8, device='cuda')
    t[:n] = torch.frombuffer(bytearray(d), dtype=torch.uint8).cuda()
    out = torch.zeros(1, dtype=torch.int64, device='cuda')
    arr = (dg._lib.Span * 1)(dg._lib.Span(0, n))
    torch.cuda.synchronize()
    ctx.check(dg.lib.dg_crc64_xz_batch_device(ctx.handle, t.data_ptr(), arr, 1, out.data_ptr(), None))
    print(n, hex(out.item() & (2**64-1)), o.crc64_xz(d).hex())
