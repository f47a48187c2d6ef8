"""Process runtime around the engines: fault injection, collective watchdog, launcher."""
from .fault import FaultSpec, parse_fault
from .watchdog import Watchdog

__all__ = ["FaultSpec", "parse_fault", "Watchdog"]
