"""GPU parity of the multi-GPU region path (kman_dgroups_*, kman_amd/dist.py)
with G simulated ranks in ONE process on one GPU (dist.SimGroup: one engine
context per rank, host-side all-reduce / all-gather, device-to-device
all-to-all).  The real run executes the same step generator with RCCL.

Bar: the ranks' outputs concatenated in rank order are bit-exact against the
numpy restatement over all shards (np_oracle: stream_kmers per shard ->
stable sort -> run-length count / uniq, seq.py:285-328, batch.py:156-168,
join.py:95-130,244-285); uniq pos carry the source rank in bits 56-63."""

from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _shards(G, nb, seed0):
    import inputs

    return [inputs.syn_numpy(nb + 997 * r, seed0 + r, record_len=50_000) for r in range(G)]


def _oracle(texts, k, mode):
    import np_oracle

    keys, pos = [], []
    for r, t in enumerate(texts):
        kk, pp = np_oracle.stream_kmers(np_oracle.parse_fasta(t), k)
        keys.append(kk)
        pos.append(pp | np.uint64(r << 56))
    keys, pos = np.concatenate(keys), np.concatenate(pos)
    sk, sp = np_oracle.stable_sort(keys, pos)
    return np_oracle.rle_count(sk) if mode == "count" else np_oracle.rle_uniq(sk, sp)


@pytest.mark.parametrize("G", [1, 2, 3, 8])
@pytest.mark.parametrize("mode", ["count", "uniq"])
@pytest.mark.parametrize("k", [15, 21])
def test_dist_region_matches_oracle(G, mode, k):
    import np_oracle  # noqa: F401
    from kman_amd import dist, engine

    texts = _shards(G, 300_000, 10 * G + k)
    devs = [engine.Device(0) for _ in range(G)]
    pipes = []
    try:
        nbq = max(sum(len(s) for _, s in __import__("np_oracle").parse_fasta(t)) for t in texts)
        for r in range(G):
            pipes.append(dist.DistPipeline(devs[r], texts[r], k, mode, G, r, None, n_bases_q=nbq))
        assert all(p.path == "region" for p in pipes)
        for _ in range(2):  # twice: the resident buffers are reused
            res = dist.SimGroup(pipes).step()
            assert all(x is not None for x in res), "a rank fell back"
            keys = np.concatenate([p.results()[0] for p in pipes])
            vals = np.concatenate([p.results()[1] for p in pipes])
            wk, wv = _oracle(texts, k, mode)
            np.testing.assert_array_equal(keys, wk)
            np.testing.assert_array_equal(vals, wv)
    finally:
        for p in pipes:
            p.free()
        for d in devs:
            d.close()
