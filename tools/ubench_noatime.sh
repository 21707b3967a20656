#!/bin/bash
# First-read cost of fresh files with and without O_NOATIME (relatime updates
# a file's atime on its first read after a write): two sets of 100K C2-sized
# files, each read once cold-in-atime by one flavour, then both again.
set -e
for S in a b; do
python3 - $S <<'PY'
import os, sys, numpy as np
d=f'/tmp/sdcas_na_{sys.argv[1]}'; os.makedirs(d, exist_ok=True)
rng=np.random.default_rng(0); buf=os.urandom(1<<17)
for i in range(100000):
    n=int(rng.integers(1024,102401))
    with open(f'{d}/{i:07d}','wb') as f: f.write(buf[:n])
PY
done
echo "first read, O_NOATIME:"; UB_NOATIME=1 timeout -k 10 120 tools/ubench_read /tmp/sdcas_na_a 100000 16 32 1 | grep pread
echo "first read, plain:";     timeout -k 10 120 tools/ubench_read /tmp/sdcas_na_b 100000 16 32 1 | grep pread
echo "second read, O_NOATIME:"; UB_NOATIME=1 timeout -k 10 120 tools/ubench_read /tmp/sdcas_na_b 100000 16 32 1 | grep pread
echo "second read, plain:";     timeout -k 10 120 tools/ubench_read /tmp/sdcas_na_a 100000 16 32 1 | grep pread
mount | grep -E " /tmp | / " | head -3 || true
rm -rf /tmp/sdcas_na_a /tmp/sdcas_na_b
