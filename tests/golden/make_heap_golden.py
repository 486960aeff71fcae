"""Extracts the heap keyed-state backend's key-group bytes of a DataStream WindowOperator from the
reference's own migration-test snapshot into a JSON fixture (tests/golden/heap_ds_reduce_event_time_flink2.2.json).

Source (paths relative to /root/reference):
  flink-streaming-java/src/test/resources/win-op-migration-test-reduce-event-time-flink2.2-snapshot
written by WindowOperatorMigrationTest.writeReducingEventTimeWindowsSnapshot
(flink-streaming-java/src/test/java/org/apache/flink/streaming/runtime/operators/windowing/
WindowOperatorMigrationTest.java:365-443): a tumbling 3 s event-time WindowOperator whose
ReducingState "window-contents" sums Tuple2<String, Integer> (SumReducer), keyed by f0 (String), in a
KeyedOneInputStreamOperatorTestHarness (max parallelism 1, one subtask: key group 0).  The restore
test (:445-514) states the continuation: watermarks 2999 / 3999 / 4999 / 5999 emit (key1, 3) and
(key2, 3) at 2999 and (key2, 2) at 5999.

This is a PURE BYTE READER: struct unpacking of the file's framing only, nothing deserialized or
executed.  The framing (OperatorSnapshotUtil.writeStateHandle, flink-runtime/src/test/java/org/apache/
flink/streaming/util/OperatorSnapshotUtil.java:48-125, with MetadataV2V3SerializerBase
.serializeKeyedStateHandle :326-348 and serializeStreamStateHandle :719-754):
  int version (3), byte NULL_HANDLE, int rawOperatorState count, int managedOperatorState count,
  int rawKeyedState count, int managedKeyedState count (1), then the managed keyed handle:
  byte KEY_GROUPS_HANDLE_V2 (12), int startKeyGroup, int numberOfKeyGroups, long offset per key
  group, then its delegate: byte BYTE_STREAM_STATE_HANDLE (1), writeUTF(name), int length, data.
The data is the heap backend's stream: the KeyedBackendSerializationProxy (KeyedBackendSerializationProxy
.java:124-138: int version 6, boolean usingKeyGroupCompression, key serializer snapshot, state meta
infos) followed by each key group at its offset (HeapSnapshotStrategy.java:161-172).  The state ids
are the meta infos' order (HeapSnapshotResources.java:100-150: ids in registration order, meta info
list in the same order); they are read here as the order of the three state names in the meta section.

Run from the repo root:  python tests/golden/make_heap_golden.py
"""
import hashlib
import json
import os
import struct
import sys

REF = "/root/reference"
SRC = "flink-streaming-java/src/test/resources/win-op-migration-test-reduce-event-time-flink2.2-snapshot"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "heap_ds_reduce_event_time_flink2.2.json")
STATE_NAMES = ["window-contents", "_timer_state/processing_window-timers", "_timer_state/event_window-timers"]


def main():
    raw = open(os.path.join(REF, SRC), "rb").read()
    at = 0

    def take(fmt):
        nonlocal at
        v = struct.unpack_from(fmt, raw, at)
        at += struct.calcsize(fmt)
        return v if len(v) > 1 else v[0]

    assert take(">i") == 3, "MetadataV3 version"
    assert take(">b") == 0, "NULL stream handle (compatibility slot)"
    raw_op, man_op, raw_keyed, man_keyed = take(">iiii")
    assert (raw_op, man_op, raw_keyed, man_keyed) == (0, 0, 0, 1), (raw_op, man_op, raw_keyed, man_keyed)
    assert take(">b") == 12, "KEY_GROUPS_HANDLE_V2"
    kg_start, n_kg = take(">ii")
    offsets = [take(">q") for _ in range(n_kg)]
    assert take(">b") == 1, "BYTE_STREAM_STATE_HANDLE"
    name_len = take(">H")
    at += name_len  # writeUTF(handle name)
    data_len = take(">i")
    data = raw[at:at + data_len]
    assert len(data) == data_len
    proxy_version, compressed = struct.unpack_from(">ib", data, 0)
    assert proxy_version == 6 and compressed == 0, "uncompressed key groups (KeyedBackendSerializationProxy v6)"
    pos = {n: data.find(n.encode()) for n in STATE_NAMES}
    assert all(p > 0 and p < offsets[0] for p in pos.values()), pos
    ids = {n: i for i, n in enumerate(sorted(STATE_NAMES, key=lambda n: pos[n]))}
    groups = []
    for i, off in enumerate(offsets):
        end = offsets[i + 1] if i + 1 < n_kg else data_len
        groups.append({"key_group": kg_start + i, "offset": off, "hex": data[off:end].hex()})
    fx = {
        "name": "ds_heap_reduce_event_time_flink2.2",
        "source": SRC,
        "source_sha256": hashlib.sha256(raw).hexdigest(),
        "writer": "WindowOperatorMigrationTest.java:365-443 (writeReducingEventTimeWindowsSnapshot)",
        "operator": {"assigner": "TumblingEventTimeWindows.of(3 s)", "trigger": "EventTimeTrigger",
                     "reduce": "SumReducer on Tuple2<String, Integer> f1 (= sum(1) keyed by f0)",
                     "key": "STRING (f0)", "record": ["STRING", "INT"], "allowed_lateness": 0,
                     "max_parallelism": kg_start + n_kg},
        "state_ids": ids,
        "key_groups": groups,
        # WindowOperatorMigrationTest.java:493-506 (testRestoreReducingEventTimeWindows)
        "continuation": [[2999, [["key1", 3, 2999], ["key2", 3, 2999]]], [3999, []], [4999, []],
                         [5999, [["key2", 2, 5999]]]],
    }
    with open(OUT, "w") as f:
        json.dump(fx, f, indent=1)
        f.write("\n")
    print(f"wrote {OUT}: key groups {[g['key_group'] for g in groups]}, ids {ids}, "
          f"{sum(len(g['hex']) // 2 for g in groups)} bytes")


if __name__ == "__main__":
    sys.exit(main())
