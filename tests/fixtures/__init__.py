"""Test fixture locations."""
import os

VENDORED = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ref")


def ref_path(rel: str) -> str:
    """A reference golden file: the vendored copy (tests/fixtures/ref, see tools/vendor_fixtures.py) if present, the
    reference mount otherwise."""
    local = os.path.join(VENDORED, rel)
    return local if os.path.exists(local) else os.path.join("/root/reference", rel)
