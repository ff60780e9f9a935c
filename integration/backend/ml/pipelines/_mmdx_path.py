"""Locates the mmdx checkout: $MMDX_HOME, else the repository these shims ship in."""
import os
import sys
from pathlib import Path

HOME = os.environ.get("MMDX_HOME") or str(Path(__file__).resolve().parents[4])
if HOME not in sys.path:
    sys.path.insert(0, HOME)
