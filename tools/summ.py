"""One-line summary of a bench.py JSON line (development): env tag, workload, events/s, ingest and
merge launch times and bytes."""
import json
import sys

tag, path = sys.argv[1], sys.argv[2]
d = json.loads(open(path).read().strip().splitlines()[-1])
r, m = d.get("roofline", {}), d.get("roofline_merge", {})
print("%-22s %-8s %6.2f G ev/s  step %.4f ms  ingest %6.1f us frac %.3f wrote %.1f MB  merge %6.1f us x%d frac %.3f read %.1f MB" % (
    tag, d["config"]["workload"].split(":")[0], d["value"] / 1e9, d["ms_per_step"], r.get("avg_launch_us", 0), r.get("frac", 0),
    r.get("partial_bytes_written_per_launch", 0) / 1e6, m.get("avg_launch_us", 0), m.get("launches", 0), m.get("frac", 0),
    m.get("partial_bytes_read_per_launch", 0) / 1e6))
