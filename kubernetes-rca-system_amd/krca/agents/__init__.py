"""Drop-in agents (ref:agents/__init__.py): same class names, constructors and analyze() contract."""
from .base import BaseAgent  # noqa: F401
from .coordinator import Coordinator  # noqa: F401
from .events import EventsAgent  # noqa: F401
from .logs import LogsAgent  # noqa: F401
from .metrics import MetricsAgent  # noqa: F401
from .resource_analyzer import ResourceAnalyzer  # noqa: F401
from .topology import TopologyAgent  # noqa: F401
from .traces import TracesAgent  # noqa: F401

__all__ = ['BaseAgent', 'MetricsAgent', 'LogsAgent', 'TracesAgent', 'TopologyAgent', 'EventsAgent',
           'Coordinator', 'ResourceAnalyzer']
