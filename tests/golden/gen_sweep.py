"""Generate tests/golden/sweep_results.json from the reference's
run_hyperparameter_sweep (eval.py:516-628) over tests/golden/sweep_small.yaml.

Test infrastructure only (build container, reference mounted read-only; the
same no-op `python-dotenv` stand-in as gen_golden.py).  The fixture is the
function's return value: the valid configurations ranked by mean on-target
ratio, with the erroring one left out.

Usage:  python tests/golden/gen_sweep.py [--out tests/golden]
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gen_golden import import_reference  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=HERE)
    args = ap.parse_args()
    import_reference()
    from quadcopter_tracking.eval import run_hyperparameter_sweep

    with tempfile.TemporaryDirectory() as tmp:
        res = run_hyperparameter_sweep(os.path.join(HERE, "sweep_small.yaml"), output_dir=tmp)
    with open(os.path.join(args.out, "sweep_results.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
