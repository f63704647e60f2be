"""Auxiliary subsystems: failure detection (watchdog), fault injection,
collective-mismatch debugging, roctx tracing and metrics logging."""
from .fault import FaultInjector  # noqa: F401
from .trace import trace_range, tracing_enabled, set_tracing  # noqa: F401
from .watchdog import Watchdog  # noqa: F401
