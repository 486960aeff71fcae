"""Mirrors of the DataStream window assigners and trigger that the GPU operator accepts.

TumblingEventTimeWindows  flink-runtime/.../windowing/assigners/TumblingEventTimeWindows.java:69-87
SlidingEventTimeWindows   flink-runtime/.../windowing/assigners/SlidingEventTimeWindows.java:77-90
EventTimeTrigger          flink-runtime/.../windowing/triggers/EventTimeTrigger.java:37-52
"""
from .._native import lib


class TumblingEventTimeWindows:
    def __init__(self, size, offset=0):
        if abs(offset) >= size or size <= 0:
            raise ValueError("TumblingEventTimeWindows parameters must satisfy abs(offset) < size")
        self.size, self.offset = size, offset

    @staticmethod
    def of(size_ms, offset_ms=0):
        return TumblingEventTimeWindows(size_ms, offset_ms)

    def assign_windows(self, timestamp):
        start = lib().fw_host_window_start(int(timestamp), self.offset % self.size, self.size)
        return [(start, start + self.size)]

    def is_event_time(self):
        return True


class SlidingEventTimeWindows:
    MAX_WINDOW_NUM = 10_000_000  # SlidingEventTimeWindows.java:50

    def __init__(self, size, slide, offset=0):
        if abs(offset) >= slide or size <= 0:
            raise ValueError("SlidingEventTimeWindows parameters must satisfy abs(offset) < slide and size > 0")
        if size // slide > self.MAX_WINDOW_NUM:
            raise ValueError("Number of windows per element exceeds MAX_WINDOW_NUM")
        self.size, self.slide, self.offset = size, slide, offset

    @staticmethod
    def of(size_ms, slide_ms, offset_ms=0):
        return SlidingEventTimeWindows(size_ms, slide_ms, offset_ms)

    def assign_windows(self, timestamp):
        last = lib().fw_host_window_start(int(timestamp), self.offset, self.slide)
        out = []
        s = last
        while s > timestamp - self.size:
            out.append((s, s + self.size))
            s -= self.slide
        return out

    def is_event_time(self):
        return True


class EventTimeTrigger:
    @staticmethod
    def create():
        return EventTimeTrigger()
