"""Drop-in for the reference's `python main_SDPL.py ...` (pseudo-label CTC objective, main_SDPL.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import suta_loader  # noqa: E402

suta_loader.load()
from suta_amd.main import main  # noqa: E402

if __name__ == "__main__":
    main(sdpl=True)
