"""The identifier dedup at BASELINE's FULL corpus sizes on one GPU, against
the oracle (file_identifier/mod.rs:149-254 inside the job's cursor steps,
file_identifier_job.rs:296-319): C3's 10 M files and C5's 50 M files in ONE
world-of-one call (sdcas_dev_dedup_local) and through the host C ABI sd-core
binds (sdcas_dedup). C5's table (2^27 u32 slots, 512 MiB) no longer fits the
256 MiB Infinity Cache, which no smaller test reaches.

Keys are real cas keys of the synthetic corpus (spacedrive_amd.synth
messages hashed on the device, a 20 000-key sample checked against upstream
BLAKE3 C); 0.2 % of the files carry an I/O error and 3000 existing Objects
(2500 of them keys the corpus carries) sit in the library. Every link and
both counts must equal the oracle's chunked dedup (oracle/cas_ref.c)."""
import importlib.util
import os

import pytest

pytestmark = pytest.mark.gpu

_spec = importlib.util.spec_from_file_location(
    "dedup_full", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "dedup_full.py"))
dedup_full = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(dedup_full)


@pytest.mark.timeout(400)
@pytest.mark.parametrize("workload", ["c3", "c5"])
def test_full_corpus_dedup_vs_oracle(workload):
    res = dedup_full.run(workload, reps=2, existing=3000, errors=0.002, parity=True, host_abi=True)
    print(res)
    assert res["files"] == dedup_full.FULL[workload] >= 10_000_000
    assert res["key_sample"]["mismatches"] == 0, res["key_sample"]
    assert res["device"]["links_equal"] and res["device"]["counts_equal"], res["device"]
    assert res["host_abi"]["links_equal"] and res["host_abi"]["counts_equal"], res["host_abi"]
    # the corpus really duplicates: C3 ~15 % duplicate files, C5 ~60 %
    created, linked = res["oracle_created_linked"]
    assert linked > (0.1 if workload == "c3" else 0.5) * res["files"], res["oracle_created_linked"]
