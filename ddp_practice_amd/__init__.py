"""ddp_practice_amd — MI355X-native single-node DDP + AMP training framework."""
import time as _time

__version__ = "0.1.0"
# wall time this interpreter first imported the package (before torch in the CLIs' ranks
# and in ddp_main.py's fork server): ddp_main.py's timer-scope check (DPA_PHASES=1)
_IMPORT_WALL = _time.time()
