"""Small helpers (reference: python/gym_ignition/utils/misc.py)."""

import tempfile


def string_to_file(string: str) -> str:
    """Write `string` to a new temporary file and return its path."""
    handle = tempfile.NamedTemporaryFile(mode="w", delete=False)
    with handle:
        handle.write(string)
    return handle.name
