"""Extracts the wire-format fixture (tests/golden/wire_fixture.json) from the reference's own test resource
flink-streaming-java/src/test/resources/win-op-migration-test-reduce-event-time-flink1.4-snapshot: the bytes of
one event-time timer of WindowOperatorMigrationTest.testRestoreReducingEventTimeWindows
(WindowOperatorMigrationTest.java:381-433, TumblingEventTimeWindows.of(3 s), key "key1", window [0, 3000)),
as the heap timer service wrote them: the key (StringSerializer: StringValue.writeString, length + 1 as a varint,
then the chars), the namespace (TimeWindow.Serializer: BE i64 start, BE i64 end) and the timestamp (BE i64
maxTimestamp = 2999).  Only bytes are read (no deserialisation).  Run here, where /root/reference exists."""
import json
import os

SRC = ("/root/reference/flink-streaming-java/src/test/resources/"
       "win-op-migration-test-reduce-event-time-flink1.4-snapshot")
HERE = os.path.dirname(os.path.abspath(__file__))

b = open(SRC, "rb").read()
i = b.find(b"\x05key1")
entry = b[i:i + 29]  # 5 string bytes + start + end + timestamp
assert entry[5:13] == bytes(8) and entry[13:21] == (3000).to_bytes(8, "big") and entry[21:29] == (2999).to_bytes(8, "big")
json.dump({"source": "flink-streaming-java/src/test/resources/win-op-migration-test-reduce-event-time-flink1.4-snapshot",
           "offset": i,
           "what": "event-time timer of key \"key1\", window [0, 3000): StringValue key, TimeWindow (BE i64 start, "
                   "BE i64 end), BE i64 timestamp 2999",
           "timer_entry_hex": entry.hex(),
           "key": "key1", "start": 0, "end": 3000, "timestamp": 2999},
          open(os.path.join(HERE, "wire_fixture.json"), "w"), indent=1)
print("wrote wire_fixture.json:", entry.hex())
