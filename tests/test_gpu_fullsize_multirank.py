"""BASELINE cfg 3, cfg 4 on 8 shards and cfg 5 at their FULL sizes, sharded
over 8 ranks (gloo, every rank on cuda:0): GLOBAL statistics against
independent per-shard counts, top-100 merges with bit-exact recomputed scores,
the 10 k-query batch merged over the shards.  See tests/fullrank.py."""
import pytest
import torch.multiprocessing as mp

import fullrank as F
import multirank as M

pytestmark = pytest.mark.gpu


def _run(tmp_path, cfg, world=8):
    out = str(tmp_path / ("%s.json" % cfg))
    mp.spawn(F.run, args=(world, M.free_port(), cfg, out), nprocs=world, join=True)
    return F.check_ranks(out, world)


def test_cfg3_10m_docs_over_8_shards_top100_and_cfg4_batch(tmp_path):
    info = _run(tmp_path, "cfg3")
    assert sum(x["docs"] for x in info) == 10_000_000
    assert all(x["term_major"] == 0 for x in info)
    assert sum(x["scores_checked"] for x in info) >= 24 * 100
    assert info[0]["batch_queries"] == 10_000


def test_cfg5_50m_short_docs_over_8_shards(tmp_path):
    info = _run(tmp_path, "cfg5")
    assert sum(x["docs"] for x in info) == 50_000_000
    assert all(x["term_major"] == 1 for x in info)
    assert info[0]["global_vocab"] > 1_000_000
