"""DataStream event-time window operator (tumbling / sliding + built-in sum/min/max) on MI355X."""
from .windowing import EventTimeTrigger, SlidingEventTimeWindows, TumblingEventTimeWindows  # noqa: F401
from .window_operator import WindowOperator, is_gpu_eligible  # noqa: F401
