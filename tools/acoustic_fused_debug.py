"""Debug aid: where do the fused and update_halo_ acoustic paths first differ?"""
import sys

import torch

sys.path.insert(0, ".")
import igg  # noqa: E402
from igg.models.acoustic2d import Acoustic2D  # noqa: E402

ny = int(sys.argv[1]) if len(sys.argv) > 1 else 48
for dtype in (torch.float32,):
    igg.init_global_grid(64, ny, 1, periodx=1, periody=0, quiet=True)
    a, b = Acoustic2D(dtype=dtype), Acoustic2D(dtype=dtype)
    assert b.set_fused(True)
    for step in range(1, 5):
        a.step()
        b.step()
        torch.cuda.synchronize()
        for n in ("P", "Vx", "Vy"):
            x, y = getattr(a, n), getattr(b, n)
            d = (x != y).nonzero()
            if d.shape[0]:
                print(dtype, "step", step, n, d.shape[0], d[:12].tolist(), flush=True)
    for n, pairs in (("Vx", [(0, 62), (64, 2)]),):
        t = getattr(b, n)
        for r0, r1 in pairs:
            print("fused", n, f"row {r0} == row {r1}:", bool(torch.equal(t[r0], t[r1])),
                  (t[r0] != t[r1]).nonzero().view(-1).tolist()[:8], flush=True)
    b.close()
    igg.finalize_global_grid()
