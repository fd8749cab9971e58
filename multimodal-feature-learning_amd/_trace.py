"""Counters of the fused / restructured paths a forward took.

Every fused autograd Function of the package counts its forward here, so a parity test can assert
that the composition it checks against the reference is the one the benchmark runs (and not a
fallback that happens to take over at the test's shapes).  Counting is a dict increment per call;
a replayed HIP graph runs no Python, so it never counts."""
import collections

hits = collections.Counter()


def hit(name, n=1):
    hits[name] += n


def clear():
    hits.clear()
