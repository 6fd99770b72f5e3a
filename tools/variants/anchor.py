"""Exact-anchor text edits for the A/B variant transforms of tools/variants/: every anchor must
occur exactly the expected number of times in the product file, or the transform exits with
status 2 (a moved anchor would otherwise build a different kernel than the one meant, or none)."""
import sys


def count_or_die(src, old, count=1, what=None):
    n = src.count(old)
    if n != count:
        sys.stderr.write(f"{sys.argv[0]}: anchor found {n} times, expected {count}: "
                         f"{what or old.strip().splitlines()[0][:100]!r}\n")
        sys.exit(2)


def replace_exact(src, old, new, count=1, what=None):
    """src with the `count` occurrences of `old` replaced; exits 2 unless there are exactly `count`."""
    count_or_die(src, old, count, what)
    return src.replace(old, new)


def index_or_die(src, anchor):
    """src.index(anchor) for an anchor that must occur exactly once; exits 2 otherwise."""
    count_or_die(src, anchor, 1)
    return src.index(anchor)
