import sys, numpy as np, torch
sys.path.insert(0, '.')
from spacedrive_amd import Engine
from spacedrive_amd.dist_dedup import DeviceStages
from tests._dist_stages import NumpyStages, make_corpus, shard
keys, has, status, existing = make_corpus(5, 2000)
(k, h, s, ids), = shard(keys, has, status, existing, 1, device="cuda")[0]
eng = Engine(); st, ns = DeviceStages(eng), NumpyStages()
rec_d, slot_d, starts_d = st.combine(k, h, s, ids, 1)
rec_n, slot_n, starts_n = ns.combine(k.cpu(), h.cpu(), s.cpu(), ids.cpu(), 1)
print('starts', starts_d, starts_n)
rd, rn = rec_d.cpu().numpy().view(np.uint64), rec_n.numpy().view(np.uint64)
print('rec shapes', rd.shape, rn.shape)
m = min(len(rd), len(rn))
bad = np.nonzero((rd[:m] != rn[:m]).any(1))[0]
print('rec mismatches', bad.size, bad[:5])
for b in bad[:5]: print(' d', [hex(x) for x in rd[b]], ' n', [hex(x) for x in rn[b]])
sd, sn = slot_d.cpu().numpy(), slot_n.numpy()
print('slot mismatches', int((sd != sn).sum()), np.nonzero(sd != sn)[0][:10], sd[:10], sn[:10])
eng.close()
