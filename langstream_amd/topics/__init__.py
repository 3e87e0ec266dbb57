"""Streaming adapters.  Importing this package registers the built-in
TopicConnectionsRuntime implementations (memory, shm, noop, kafka, pulsar, pravega)."""
from . import memory  # noqa: F401
from . import shm  # noqa: F401
try:  # optional adapters register themselves when importable
    from . import kafka  # noqa: F401
except ImportError:  # pragma: no cover
    pass
try:
    from . import pulsar  # noqa: F401
except ImportError:  # pragma: no cover
    pass
try:
    from . import pravega  # noqa: F401
except ImportError:  # pragma: no cover
    pass
