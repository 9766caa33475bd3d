"""Agent interface of the drop-in boundary.

Mirrors ``BaseAgent`` of the reference (ref:agents/base_agent.py:1-84): constructor takes the
duck-typed cluster client, ``analyze(namespace, context=None, **kwargs)`` returns
``{'findings', 'reasoning_steps'[, 'error'][, additive keys]}``, findings/steps carry the
client's ``get_current_time()`` stamp.  Agents are stateful and single-threaded exactly like
the reference (state is reset at the start of every ``analyze``).
"""

SEVERITY_ORDER = ("info", "low", "medium", "high", "critical")  # ref:agents/coordinator.py:150


class BaseAgent:
    """Common findings / reasoning accumulators (ref:agents/base_agent.py:7-84)."""

    def __init__(self, k8s_client, engine=None):
        self.k8s_client = k8s_client
        self._engine = engine
        self.findings = []
        self.reasoning_steps = []

    # -- engine: the MI355X numeric core behind this agent (no CPU fallback) -------------
    @property
    def engine(self):
        if self._engine is None:
            from krca import native
            self._engine = native.default_engine()
        return self._engine

    def analyze(self, namespace, context=None, **kwargs):  # ref:agents/base_agent.py:18-31
        raise NotImplementedError("Each agent must implement its own analyze method")

    def add_finding(self, component, issue, severity, evidence, recommendation):
        self.findings.append(dict(component=component, issue=issue, severity=severity,
                                  evidence=evidence, recommendation=recommendation,
                                  timestamp=self.k8s_client.get_current_time()))

    def add_reasoning_step(self, observation, conclusion):
        self.reasoning_steps.append(dict(observation=observation, conclusion=conclusion,
                                         timestamp=self.k8s_client.get_current_time()))

    def get_results(self):
        return {"findings": self.findings, "reasoning_steps": self.reasoning_steps}

    def reset(self):
        self.findings = []
        self.reasoning_steps = []

    # shared error contract of every analyze() (e.g. ref:agents/metrics_agent.py:58-67)
    def _error_result(self, what, exc):
        self.add_reasoning_step(observation=f"Error occurred during {what} analysis: {str(exc)}",
                                conclusion=f"Unable to complete {what} analysis due to an error")
        return {"error": str(exc), "findings": self.findings, "reasoning_steps": self.reasoning_steps}

    def _maybe_set_context(self, context):
        if context:
            self.k8s_client.set_context(context)
