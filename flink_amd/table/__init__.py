"""Table/SQL window TVF aggregation (TUMBLE / HOP / CUMULATE) on MI355X."""
from .slice_assigners import SliceAssigners  # noqa: F401
from .window_agg import WindowAggOperator, is_gpu_eligible  # noqa: F401
