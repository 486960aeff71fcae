"""Mirror of SliceAssigners (flink-table-runtime/.../operators/window/tvf/slicing/SliceAssigners.java).

The assigner objects describe the window for the GPU operator and expose the reference's
scalar slice arithmetic on the host (window_start goes through the library's host entry point,
i.e. the exact code the kernels run).  Event time.  A TIMESTAMP_LTZ window carries its shift time
zone (SliceAssigners.tumbling/hopping/cumulative(rowtimeIndex, shiftTimeZone, ...)): rowtimes are
sliced on the zone's wall clock (AbstractSliceAssigner.assignSliceEnd :655-670), DST included.
"""
import math

from .. import abi
from .._native import lib


def _window_start(ts, offset, size):
    return lib().fw_host_window_start(int(ts), int(offset), int(size))


class SliceAssigner:
    kind = None
    shared = False

    shift_zone = None  # flink_amd.table.time_zone.ShiftZone, None = UTC

    def __init__(self, rowtime_index, size, slide, offset):
        self.rowtime_index = rowtime_index
        self.size = size
        self.slide = slide
        self.offset = offset

    def in_zone(self, zone):
        """The same assigner on a TIMESTAMP_LTZ rowtime sliced in `zone` (name or ShiftZone)."""
        import copy
        from .time_zone import ShiftZone
        a = copy.copy(self)
        a.shift_zone = ShiftZone.of(zone) if isinstance(zone, str) else zone
        return a

    def get_slice_end_interval(self):
        raise NotImplementedError

    def assign_slice_end(self, timestamp):
        iv = self.get_slice_end_interval()
        if self.shift_zone is not None:  # toUtcTimestampMills (TimeWindowUtil.java:52-60)
            timestamp = self.shift_zone.to_utc_timestamp_mills(timestamp)
        return _window_start(timestamp, self.offset, iv) + iv

    def is_event_time(self):
        return self.rowtime_index >= 0


class TumblingSliceAssigner(SliceAssigner):
    """SliceAssigners.TumblingSliceAssigner (:140-200)."""
    kind = abi.WIN_TUMBLE

    def __init__(self, rowtime_index, size, offset=0):
        if size <= 0:
            raise ValueError(f"Tumbling Window parameters must satisfy size > 0, but got size {size}ms.")
        if abs(offset) >= size:
            raise ValueError(f"Tumbling Window parameters must satisfy abs(offset) < size, but got size {size}ms and offset {offset}ms.")
        super().__init__(rowtime_index, size, 0, offset)

    def with_offset(self, offset):
        return TumblingSliceAssigner(self.rowtime_index, self.size, offset)

    def get_slice_end_interval(self):
        return self.size

    def get_last_window_end(self, slice_end):
        return slice_end

    def get_window_start(self, window_end):
        return window_end - self.size

    def expired_slices(self, window_end):
        return [window_end]


class HoppingSliceAssigner(SliceAssigner):
    """SliceAssigners.HoppingSliceAssigner (:203-316); slices of gcd(size, slide)."""
    kind = abi.WIN_HOP
    shared = True

    def __init__(self, rowtime_index, size, slide, offset=0):
        if size <= 0 or slide <= 0:
            raise ValueError(f"Hopping Window must satisfy slide > 0 and size > 0, but got slide {slide}ms and size {size}ms.")
        if size % slide != 0:
            raise ValueError(f"Slicing Hopping Window requires size must be an integral multiple of slide, but got size {size}ms and slide {slide}ms.")
        super().__init__(rowtime_index, size, slide, offset)
        self.slice_size = math.gcd(size, slide)
        self.num_slices_per_window = size // self.slice_size

    def with_offset(self, offset):
        return HoppingSliceAssigner(self.rowtime_index, self.size, self.slide, offset)

    def get_slice_end_interval(self):
        return self.slice_size

    def get_last_window_end(self, slice_end):
        return slice_end - self.slice_size + self.size

    def get_window_start(self, window_end):
        return window_end - self.size

    def expired_slices(self, window_end):
        return [self.get_window_start(window_end) + self.slice_size]

    def slices_to_merge(self, window_end):
        """HoppingSlicesIterable: n slices ending at window_end, newest first; null target."""
        return None, [window_end - i * self.slice_size for i in range(self.num_slices_per_window)]

    def next_trigger_window(self, window_end, is_window_empty):
        """HoppingSliceAssigner.nextTriggerWindow: the next window while this one is not empty."""
        return None if is_window_empty else window_end + self.slice_size


class CumulativeSliceAssigner(SliceAssigner):
    """SliceAssigners.CumulativeSliceAssigner (:319-454)."""
    kind = abi.WIN_CUMULATE
    shared = True

    def __init__(self, rowtime_index, max_size, step, offset=0):
        if max_size <= 0 or step <= 0:
            raise ValueError(f"Cumulative Window parameters must satisfy maxSize > 0 and step > 0, but got maxSize {max_size}ms and step {step}ms.")
        if max_size % step != 0:
            raise ValueError(f"Cumulative Window requires maxSize must be an integral multiple of step, but got maxSize {max_size}ms and step {step}ms.")
        super().__init__(rowtime_index, max_size, step, offset)

    def with_offset(self, offset):
        return CumulativeSliceAssigner(self.rowtime_index, self.size, self.slide, offset)

    def get_slice_end_interval(self):
        return self.slide

    def get_window_start(self, window_end):
        return _window_start(window_end - 1, self.offset, self.size)

    def get_last_window_end(self, slice_end):
        return self.get_window_start(slice_end) + self.size

    def expired_slices(self, window_end):
        ws = self.get_window_start(window_end)
        first, last = ws + self.slide, ws + self.size
        if window_end == first:
            return []
        if window_end == last:
            return [window_end, first]
        return [window_end]

    def slices_to_merge(self, window_end):
        first = self.get_window_start(window_end) + self.slide
        return first, ([] if window_end == first else [window_end])

    def next_trigger_window(self, window_end, is_window_empty):
        """CumulativeSliceAssigner.nextTriggerWindow: the next step up to the window's max size,
        empty or not."""
        nxt = window_end + self.slide
        return None if nxt > self.get_window_start(window_end) + self.size else nxt


class SliceAssigners:
    """Factory methods with the reference's names (durations in milliseconds)."""

    @staticmethod
    def tumbling(rowtime_index, size_ms):
        return TumblingSliceAssigner(rowtime_index, size_ms)

    @staticmethod
    def hopping(rowtime_index, size_ms, slide_ms):
        return HoppingSliceAssigner(rowtime_index, size_ms, slide_ms)

    @staticmethod
    def cumulative(rowtime_index, max_size_ms, step_ms):
        return CumulativeSliceAssigner(rowtime_index, max_size_ms, step_ms)
