"""End to end on the reference's own real-data fixture
(static/datasets/preprocessing_example/s2cs_tiny_preproc.parquet: 326 documents,
columns id / bow_text / fos / embeddings[192]).  The reference ships no outputs
for it, so model numbers are "parity unpinned"; what is pinned is the protocol:
the vocabulary consensus equals the reference recipe (per-client
CountVectorizer(lowercase, stop_words='english'), sorted union; client.py:369-374,
server.py:270-279) and every client trains on its own field of study."""
import os

import numpy as np
import pytest

FIXTURE = "/root/reference/static/datasets/preprocessing_example/s2cs_tiny_preproc.parquet"
pytestmark = pytest.mark.skipif(not os.path.exists(FIXTURE), reason="reference fixture absent")

FOS = ["computer_science", "economics", "sociology", "political_science", "philosophy"]


def _params(**kw):
    from gfedntm_amd.utils.config import load_config
    p = dict(load_config().training_params)
    p.update(num_epochs=2, batch_size=16, n_components=5, hidden_sizes=(16, 16))
    p.update(kw)
    return p


def test_consensus_matches_reference_recipe_and_avitm_trains():
    import pandas as pd
    from sklearn.feature_extraction.text import CountVectorizer
    from gfedntm_amd.federation.data import load_client_corpus
    from gfedntm_amd.federation.runner import LocalFederation
    corpora = [load_client_corpus("real", FIXTURE, i + 1, fos=f) for i, f in enumerate(FOS)]
    df = pd.read_parquet(FIXTURE)
    ref_union = set()
    for f in FOS:
        texts = df[df.fos == f].bow_text.tolist()
        ref_union |= set(CountVectorizer(lowercase=True, stop_words="english").fit(texts).vocabulary_)
    fed = LocalFederation(corpora, _params(), max_iters=12, device="cpu", backend="torch", seed=0)
    assert fed.terms == sorted(ref_union)
    assert [c.n_docs for c in fed.clients] == [int((df.fos == f).sum()) for f in FOS]
    fed.run()
    h = np.stack([c.loss_history()[:12] for c in fed.clients])
    assert np.isfinite(h).all()
    a = fed.clients[0].shared
    assert all(bool((c.shared == a).all()) for c in fed.clients[1:])


def test_combined_tm_on_fixture_embeddings():
    from gfedntm_amd.federation.data import load_client_corpus
    from gfedntm_amd.federation.runner import LocalFederation
    corpora = [load_client_corpus("real", FIXTURE, i + 1, fos=f) for i, f in enumerate(FOS[:3])]
    assert corpora[0].embeddings.shape[1] == 192
    fed = LocalFederation(corpora, _params(contextual_size=192), model_type="ctm", max_iters=8,
                          device="cpu", backend="torch", seed=0)
    fed.run()
    for c in fed.clients:
        betas, thetas, topics = c.results()
        assert betas.shape == (5, len(fed.terms)) and thetas.shape[0] == c.n_docs
        assert len(topics) == 5 and all(len(t) == 10 for t in topics)
