"""User-facing Python agent API (source-compatible with the reference's ``langstream``
package, RTPY/langstream/api.py:30-199): implement Source / Processor / Sink / Service
and reference the class with ``className`` in a python-* agent.  Agents run
in-process in the MI355X runtime (no gRPC sidecar)."""
from .api import Agent, AgentContext, Processor, Record, RecordType, Service, Sink, Source
from .util import AvroValue, SimpleRecord

__all__ = ["Record", "RecordType", "Agent", "Source", "Sink", "Processor", "Service", "SimpleRecord", "AvroValue",
           "AgentContext"]
