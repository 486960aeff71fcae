"""Shift time zones of TIMESTAMP_LTZ windows (TimeWindowUtil.getShiftTimeZone,
flink-table/flink-table-runtime/.../util/TimeWindowUtil.java:163-167).

A window on a TIMESTAMP_LTZ rowtime is sliced on the zone's local wall clock: the slice assigner
converts each epoch rowtime with toUtcTimestampMills (:52-60), and window timers go back to epoch
time with toEpochMillsForTimer (:69-140).  The device evaluates both from a piecewise-constant
offset table: ``utc[i]`` is the UTC instant (epoch ms) from which ``offset_ms[i]`` is in force
(``utc[0]`` = Long.MIN_VALUE), i.e. java.time ZoneRules.getOffset(Instant) expanded over a year
range.  The Java shim builds the table from ZoneRules.getTransitions() +
getTransitionRules(); this host mirror builds it from the IANA database through ``zoneinfo`` by
locating every offset change (day scan, then bisection to the second), which gives the same
transitions for the same tzdata version.
"""
import datetime as _dt
import functools
from dataclasses import dataclass

INT64_MIN = -(1 << 63)
_DAY = 86400


@dataclass(frozen=True)
class ShiftZone:
    name: str
    utc: tuple          # ascending UTC epoch ms, utc[0] = INT64_MIN
    offset_ms: tuple    # offset in force from utc[i]
    use_dst: bool       # TimeZone.getTimeZone(zone).useDaylightTime()

    @staticmethod
    @functools.lru_cache(maxsize=None)
    def of(name, first_year=1900, last_year=2100):
        if name in ("UTC", "Z", "GMT"):
            return ShiftZone(name, (INT64_MIN,), (0,), False)
        from zoneinfo import ZoneInfo
        tz = ZoneInfo(name)

        def off(sec):
            return int(_dt.datetime.fromtimestamp(sec, tz).utcoffset().total_seconds())

        lo = int(_dt.datetime(first_year, 1, 1, tzinfo=_dt.timezone.utc).timestamp())
        hi = int(_dt.datetime(last_year, 12, 31, tzinfo=_dt.timezone.utc).timestamp())
        utc, offs = [INT64_MIN], [off(lo) * 1000]
        prev_t, prev = lo, off(lo)
        for t in range(lo + _DAY, hi, _DAY):
            o = off(t)
            if o == prev:
                prev_t = t
                continue
            a, b = prev_t, t  # off(a) == prev != off(b): the change is in (a, b]
            while b - a > 1:
                m = (a + b) // 2
                if off(m) == prev:
                    a = m
                else:
                    b = m
            utc.append(b * 1000)
            offs.append(o * 1000)
            prev_t, prev = t, o
        # useDaylightTime(): the zone observes daylight saving now or in the future (java.util
        # .TimeZone over ZoneRules: a DST transition rule or a DST offset after the current year)
        this_year = int(_dt.datetime(_dt.datetime.now(_dt.timezone.utc).year, 1, 1,
                                     tzinfo=_dt.timezone.utc).timestamp()) * 1000
        use_dst = sum(1 for u in utc[1:] if u >= this_year) >= 2
        return ShiftZone(name, tuple(utc), tuple(offs), use_dst)

    # -- host restatements (used by the API layer and tests) --------------------------------
    def offset_at(self, epoch_ms):
        import bisect
        return self.offset_ms[bisect.bisect_right(self.utc, epoch_ms) - 1]

    def to_utc_timestamp_mills(self, epoch_ms):
        """TimeWindowUtil.toUtcTimestampMills."""
        if epoch_ms == (1 << 63) - 1:
            return epoch_ms
        return epoch_ms + self.offset_at(epoch_ms)
