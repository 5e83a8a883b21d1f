#!/usr/bin/env python3
"""Randomised LIVE parity sweep from the command line (the sweep itself is tests/ref_sweep.py).
python fuzz_ref.py [cases] [seed] [m_n_lo:m_n_hi k_lo:k_hi]
Environment: FUZZ_EXTREME=1 (half the cases with extreme / non-finite inputs), FUZZ_AB=general (complex and
general alpha, beta), FUZZ_LD=1 (padded leading dimensions), FUZZ_REF_EPI=1 (reference-epilogue mode),
FUZZ_OUT (file name under gpurun_out/, default fuzz_ref.json)."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "mixed-gemmul8_amd")]
from ref_sweep import COMBOS, NPT, TDT_NAMES, defect, sweep  # noqa: E402,F401  (re-exported for the other probes)

TDT = {t: getattr(torch, name) for t, name in TDT_NAMES.items()}


def main():
    cases = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    mn = kr = None
    if len(sys.argv) > 4:  # size ranges: m, n in [a, b), k in [c, d)
        mn, kr = tuple(map(int, sys.argv[3].split(":"))), tuple(map(int, sys.argv[4].split(":")))
    t0 = time.time()
    out = sweep(cases, seed, mn, kr, extreme=os.environ.get("FUZZ_EXTREME") == "1",
                ab_mode=os.environ.get("FUZZ_AB", "basic"), ld=os.environ.get("FUZZ_LD") == "1",
                ref_epi=os.environ.get("FUZZ_REF_EPI") == "1")
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", os.environ.get("FUZZ_OUT", "fuzz_ref.json")), "w") as f:
        json.dump(out, f, indent=1)
    print(f"{out['cases']} cases, {len(out['failures'])} failures, {len(out['outputs_left_unchanged'])} outputs "
          f"unchanged, {out['differ_only_in_nonfinite_vectors']} differ only in rows / columns with non-finite "
          f"inputs, skipped {out['skipped_defect_classes']}, {time.time() - t0:.0f} s", flush=True)
    sys.exit(1 if out["failures"] else 0)


if __name__ == "__main__":
    main()
