"""``python -m nightcore_analyzer``: the reference launches its PyQt6 GUI here
(__main__.py:11-39).  The GUI is out of this engine's scope; run the CLI."""
import sys

from .cli import main

if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
