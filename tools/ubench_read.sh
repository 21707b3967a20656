#!/bin/bash
# host read-rate probe: 200K C2-sized files in /tmp, pread vs io_uring
set -e
D=/tmp/sdcas_ur
python3 - <<'PY'
import os, numpy as np
d='/tmp/sdcas_ur'; os.makedirs(d, exist_ok=True)
rng=np.random.default_rng(0); buf=os.urandom(1<<17)
for i in range(200000):
    n=int(rng.integers(1024,102401))
    with open(f'{d}/{i:07d}','wb') as f: f.write(buf[:n])
PY
for T in 4 8 16; do timeout -k 10 120 tools/ubench_read $D 200000 $T 32 2; done
timeout -k 10 120 tools/ubench_read $D 200000 16 64 2
rm -rf $D
