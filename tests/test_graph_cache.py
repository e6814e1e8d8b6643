"""Per-lane graph cache of HipGPT (engine.py _cached_graph / _keep_graph / _drop_graphs): a lane keeps the graphs
it captured for each (path, shape) key, so alternating between the persistent layers and the launch chain for the
same shape (synthesize_many's overlap) replays instead of recapturing.  Host logic only: the "graphs" are tokens."""
from indextts.gpt.engine import HipGPT


class _Eng:
    GRAPH_CACHE = HipGPT.GRAPH_CACHE
    _keep_graph = HipGPT._keep_graph
    _cached_graph = HipGPT._cached_graph
    _drop_graphs = staticmethod(HipGPT._drop_graphs)


def test_alternating_keys_capture_once_each():
    eng, ln, captured = _Eng(), {"graph": None}, []

    def cap(tag):
        def f():
            captured.append(tag)
            return tag
        return f

    for _ in range(3):  # persistent layers, then the chain, for the same shape, three times over
        assert eng._cached_graph(ln, ("pl", 32), cap("pl")) == "pl"
        assert eng._cached_graph(ln, ("chain", 32), cap("chain")) == "chain"
    assert captured == ["pl", "chain"]


def test_cache_is_bounded_and_drop_clears_it():
    eng, ln = _Eng(), {"graph": None}
    for i in range(eng.GRAPH_CACHE + 3):
        eng._cached_graph(ln, i, lambda i=i: i)
    assert len(ln["graphs"]) == eng.GRAPH_CACHE
    assert ("one", 0) not in ln["graphs"] and ("one", eng.GRAPH_CACHE + 2) in ln["graphs"]  # oldest evicted first
    eng._drop_graphs(ln)
    assert ln["graphs"] == {} and ln["graph"] is None and ln["multi"] is None
