"""Width-tagged numbers.

Python has one ``int`` and one ``float``; the reference's records carry Java boxed types
(Short / Integer / Long, Float / Double) whose Kafka serialisers write 2 / 4 / 8 and 4 / 8
big-endian bytes (KRT/KafkaProducerWrapper.java:57-67).  The compute / cast steps tag
their results with these subclasses (INT8 / INT16 / INT32 / FLOAT) so a value typed INT32
in the pipeline leaves on a topic as 4 bytes, exactly as the Java runtime writes it.
They behave as plain ints / floats everywhere else.  An untagged int is a Long, an
untagged float a Double (what the reference's Python bridge maps them to,
RTPY/langstream_grpc/grpc_service.py:294-305)."""
from __future__ import annotations


class Int8(int):
    java = "Byte"


class Int16(int):
    java = "Short"


class Int32(int):
    java = "Integer"


class Float32(float):
    java = "Float"
