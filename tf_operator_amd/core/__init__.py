"""Python face of the C++17 operator core (``_toa_core``, csrc/core/)."""
from __future__ import annotations

import importlib


def native():
    """Return the compiled pybind11 module; raise if it has not been built."""
    try:
        return importlib.import_module("tf_operator_amd.core._toa_core")
    except ImportError as e:  # pragma: no cover
        raise RuntimeError("C++ operator core not built: run `python -m tf_operator_amd._build --only core`") from e
