"""Synthetic corpora of SURVEY.md §8d (configs C2, C3, C4, C5) as (size,
content key) per file — the numpy side of include/sdcas_synth.h.

packages/test-files (config C1) is empty in the reference snapshot, so every
workload is generated. A file is (size, content key); its bytes are
sds_content_word(key, w) (include/sdcas_synth.h), generated straight into HBM
by sdcas_dev_synth_cas_messages / sdcas_dev_synth_content. Duplicate files
share a content id and therefore size and key. Workload definition only —
nothing here hashes.
"""
import numpy as np

SEED_C2, SEED_C3, SEED_C4, SEED_C5 = 0x5D0002, 0x5D0003, 0x5D0004, 0x5D0005
MIN_FILE = 102400            # cas.rs:15 MINIMUM_FILE_SIZE
SAMPLED_MSG_LEN = 57352      # le64 + 8 KiB header + 4 x 10 KiB samples + 8 KiB footer

_U = np.uint64


def mix64(x):
    with np.errstate(over="ignore"):
        z = np.asarray(x, dtype=_U) + _U(0x9E3779B97F4A7C15)
        z = (z ^ (z >> _U(30))) * _U(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> _U(27))) * _U(0x94D049BB133111EB)
        return z ^ (z >> _U(31))


def content_key(seed, cid):
    """sds_content_key(seed, content_id)"""
    with np.errstate(over="ignore"):
        return mix64(_U(seed) ^ (np.asarray(cid, dtype=_U) * _U(0xD1B54A32D192ED03)))


def unit(r):
    """uniform [0, 1) doubles from the top 53 bits of u64 randoms"""
    return (np.asarray(r, dtype=_U) >> _U(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def cas_msg_len(sizes):
    """sds_cas_msg_len: whole-file (cas.rs:27-29) or sampled (cas.rs:30-59)"""
    s = np.asarray(sizes, dtype=_U)
    return np.where(s <= _U(MIN_FILE), s + _U(8), _U(SAMPLED_MSG_LEN)).astype(_U)


def c2_files(lo, hi, seed=SEED_C2):
    """C2: size ~ Uniform{1024..102400}, content id = file index (sds_c2_size)"""
    i = np.arange(lo, hi, dtype=_U)
    with np.errstate(over="ignore"):
        raw = mix64(_U(seed) ^ _U(0xC2C2C2C2) ^ (i << _U(20)) ^ (i >> _U(44)))
    sizes = _U(1024) + raw % _U(102400 - 1024 + 1)
    return sizes, content_key(seed, i)


def _log_uniform(r, lo, hi):
    """integer size in [lo, hi], log-uniform"""
    x = np.exp(np.log(lo) + unit(r) * (np.log(hi + 1.0) - np.log(lo)))
    return np.clip(np.floor(x), lo, hi).astype(_U)


def c3_content_ids(hi, seed=SEED_C3, dup_frac=0.15):
    """content id of files [0, hi): 15% of files (index > 0) duplicate a
    uniformly chosen earlier file, chased to that file's own content"""
    i = np.arange(hi, dtype=_U)
    with np.errstate(over="ignore"):
        r = mix64(_U(seed) ^ _U(0xD0D0D0D0) ^ (i * _U(0x9FB21C651E98DF25)))
    dup = (unit(r) < dup_frac) & (i > 0)
    src = (unit(mix64(r)) * i.astype(np.float64)).astype(np.int64)
    cid = np.where(dup, src, np.arange(hi, dtype=np.int64))
    while True:  # src < i, so chasing converges in O(log) rounds
        nxt = cid[cid]
        if np.array_equal(nxt, cid):
            return cid.astype(_U)
        cid = nxt


def c3_sizes_of(cid, seed=SEED_C3):
    """75% whole-file: log-uniform [1 B, 100 KiB]; 25% sampled: log-uniform
    (100 KiB, 64 GiB] (only the hashed windows are ever materialised)"""
    r = mix64(_U(seed) ^ _U(0x512E512E) ^ np.asarray(cid, dtype=_U))
    sampled = (r & _U(3)) == _U(0)
    r2 = mix64(r)
    small = _log_uniform(r2, 1.0, float(MIN_FILE))
    big = _log_uniform(r2, float(MIN_FILE + 1), float(64 << 30))
    return np.where(sampled, big, small)


def c3_files(lo, hi, seed=SEED_C3):
    cid = c3_content_ids(hi, seed)[lo:hi]
    return c3_sizes_of(cid, seed), content_key(seed, cid), cid


def c5_content_ids(lo, hi, seed=SEED_C5, distinct=20_000_000, s=1.1):
    return c5_content_ids_at(np.arange(lo, hi, dtype=_U), seed, distinct, s)


def c5_content_ids_at(i, seed=SEED_C5, distinct=20_000_000, s=1.1):
    """files [0, distinct) own contents [0, distinct); the rest draw a
    content id from Zipf(s) over `distinct` (inverse-CDF on the continuous
    approximation, rank 1 = content 0)"""
    i = np.asarray(i, dtype=_U)
    r = mix64(_U(seed) ^ _U(0x21FF21FF) ^ i)
    u = unit(r)
    # continuous Zipf on [1, N+1): CDF(x) = (1 - x^(1-s)) / (1 - (N+1)^(1-s))
    a = 1.0 - s
    x = (1.0 - u * (1.0 - (distinct + 1.0) ** a)) ** (1.0 / a)
    z = np.clip(np.floor(x) - 1, 0, distinct - 1).astype(_U)
    return np.where(i < _U(distinct), i, z)


def c5_sizes_of(cid, seed=SEED_C5, lo=1024.0, hi=float(1 << 30), alpha=1.1):
    """bounded Pareto(alpha) on [1 KiB, 1 GiB] per content"""
    u = unit(mix64(_U(seed) ^ _U(0x9A9A9A9A) ^ np.asarray(cid, dtype=_U)))
    la, ha = lo ** alpha, hi ** alpha
    x = (-(u * ha - u * la - ha) / (ha * la)) ** (-1.0 / alpha)
    return np.clip(np.floor(x), lo, hi).astype(_U)


def c5_files(lo, hi, seed=SEED_C5, distinct=20_000_000):
    cid = c5_content_ids(lo, hi, seed, distinct)
    return c5_sizes_of(cid, seed), content_key(seed, cid), cid


def c4_files(total_bytes=256 << 30, seed=SEED_C4):
    """C4: sizes ~ Uniform{2^30 .. 2^32} drawn until their sum reaches
    total_bytes (the last one truncated); content id = file index"""
    sizes = []
    acc, i = 0, 0
    while acc < total_bytes:
        r = int(mix64(_U(seed) ^ _U(0xC4C4C4C4) ^ _U(i)))
        s = (1 << 30) + r % ((1 << 32) - (1 << 30) + 1)
        s = min(s, total_bytes - acc)
        sizes.append(s)
        acc += s
        i += 1
    sizes = np.array(sizes, dtype=_U)
    return sizes, content_key(seed, np.arange(sizes.size, dtype=_U))
