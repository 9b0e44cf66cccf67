#!/usr/bin/env python3
"""varbin.py drop-in (binning.sh:36: `$SMASH_CODE/varbin.py POSITIONS BINS
OUT STATS CHROM_SIZES`): the same five arguments and outputs as the
reference's varbin.py (varbin.py:6-118), with the counting loop (adjacent
de-dup, bisect_right, counts) on the device through libsmashgpu
(smash_bin_positions); see smash_cli.cmd_varbin."""
import os
import sys

HERE = os.path.dirname(os.path.realpath(__file__))
for p in (os.path.join(HERE, ".."), HERE):
    if os.path.exists(os.path.join(p, "smash_cli.py")):
        sys.path.insert(0, p)
        break
import smash_cli  # noqa: E402

if __name__ == "__main__":
    if len(sys.argv) != 6:
        raise SystemExit("usage: varbin.py positions bins out stats chrom_sizes")
    smash_cli.main(["varbin"] + sys.argv[1:])
