"""Pins the golden zipf draws to the REFERENCE's generator (run from repo
root: `python tests/golden/make_zipf_ref.py [--write]`).

Builds oracle/_ref/zipf_ref (`make -C oracle ref`: the reference's own
test/zipf.h compiled by path from /root/reference with -ffp-contract=off and
a driver of ours, oracle/zipf_ref_main.cpp), draws 256 values for every
(n, theta, seed) of tests/golden/generators.json, and checks them against
the fixture (the oracle's restatement, make_golden.py) — with --write it
stores the reference's draws into the fixture instead.  Exit status 0 = the
fixture equals the reference's output."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
FIX = os.path.join(ROOT, "tests", "golden", "generators.json")
BIN = os.path.join(ROOT, "oracle", "_ref", "zipf_ref")


def reference_draws(n, theta, seed, count):
    out = subprocess.run([BIN, str(n), repr(float(theta)), str(seed), str(count)],
                         capture_output=True, text=True, check=True).stdout
    return [int(x) for x in out.split()]


def main():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "ref"])
    gen = json.load(open(FIX))
    ok = True
    for z in gen["zipf"]:
        ref = reference_draws(z["n"], z["theta"], z["seed"], len(z["draws"]))
        same = ref == z["draws"]
        print(f"n={z['n']} theta={z['theta']} seed={z['seed']:#x}: "
              f"{'equal' if same else 'DIFFERENT'}")
        ok = ok and same
        z["draws"] = ref
    if "--write" in sys.argv:
        with open(FIX, "w") as f:
            json.dump(gen, f)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
