"""Where workgroups land: HW_ID / XCC_ID of a grid of spinning workgroups (the CU
topology behind any CU-reservation scheme)."""
import collections
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sparsecholesky_amd as sc  # noqa: E402

for nwg, thr in ((256, 512), (2048, 256)):
    out = np.zeros(2 * nwg, dtype=np.uint32)
    assert sc.lib().sc_debug_hwid(nwg, thr, 20000, out.ctypes.data) == 0
    hw, xcc = out[0::2], out[1::2] & 0xF
    cu, sh, se = (hw >> 8) & 0xF, (hw >> 12) & 0x1, (hw >> 13) & 0x7
    keys = collections.Counter(zip(xcc.tolist(), se.tolist(), sh.tolist(), cu.tolist()))
    print(f"{nwg} wgs x {thr}: distinct (xcc,se,sh,cu) {len(keys)}; xcc {sorted(set(xcc.tolist()))}; "
          f"se {sorted(set(se.tolist()))}; sh {sorted(set(sh.tolist()))}; cu {sorted(set(cu.tolist()))}")
    print("  per-xcc distinct CUs:", {x: len({k for k in keys if k[0] == x}) for x in sorted(set(xcc.tolist()))})
    print("  first 16 (wg -> xcc,se,sh,cu):", [(i, int(xcc[i]), int(se[i]), int(sh[i]), int(cu[i])) for i in range(16)])
