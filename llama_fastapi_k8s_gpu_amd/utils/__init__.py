"""Small shared utilities: timers and rocprofv3 result summaries."""
from .timing import Timer, percentile  # noqa: F401
