"""TracesAgent (host): tracing-platform detection and the reference's simulated findings.

Reference: ref:agents/traces_agent.py:3-381 — no data arithmetic (its latency/error/dependency
findings are canned, :209-381).  Out of the hot-path scope; kept so the comprehensive run
correlates identical finding lists.
"""
from .base import BaseAgent

_TRACE_KEYS = ('jaeger', 'zipkin', 'tracing', 'otel', 'opentelemetry')


class TracesAgent(BaseAgent):
    def analyze(self, namespace, context=None, **kwargs):
        self.reset()
        try:
            self._maybe_set_context(context)
            found = {p: self._platform(p) for p in ('jaeger', 'zipkin', 'opentelemetry')}
            if not any(found.values()):
                self.add_reasoning_step(observation="No distributed tracing platform detected in the cluster",
                                        conclusion="Unable to analyze traces without a tracing platform")
                self.add_finding(component="Tracing Infrastructure", issue="No distributed tracing platform detected",
                                 severity="medium", evidence="No Jaeger, Zipkin, or OpenTelemetry collectors found",
                                 recommendation="Deploy a distributed tracing solution like Jaeger or OpenTelemetry to enable trace analysis")
                self._instrumented(namespace)
                return self.get_results()
            platform = next(p for p in ('jaeger', 'zipkin', 'opentelemetry') if found[p])
            self.add_reasoning_step(observation=f"Detected {platform} tracing platform",
                                    conclusion="Will analyze trace data from this platform")
            svcs = self._instrumented(namespace)
            if not svcs:
                self.add_reasoning_step(
                    observation=f"No services in namespace {namespace} appear to be instrumented for tracing",
                    conclusion="Unable to analyze traces without instrumented services")
                self.add_finding(component="Service Instrumentation",
                                 issue=f"No services in namespace {namespace} appear to be instrumented for tracing",
                                 severity="medium",
                                 evidence="No tracing environment variables or configuration detected in deployments",
                                 recommendation="Instrument your services for distributed tracing to enable cross-service request analysis")
                return self.get_results()
            self._simulated(svcs)
            return self.get_results()
        except Exception as e:
            return self._error_result("traces", e)

    def _platform(self, name):  # ref :118-146
        try:
            hits = [self.k8s_client.get_services_by_label(f'app={name}{suffix}')
                    for suffix in ('', '-collector', '-query')]
            return any(len(h) > 0 for h in hits)
        except Exception as e:
            self.add_reasoning_step(observation=f"Error checking for {name}: {str(e)}",
                                    conclusion=f"Unable to determine if {name} is deployed")
            return False

    def _instrumented(self, namespace):  # ref :148-207
        out = []
        try:
            for d in self.k8s_client.get_deployments(namespace):
                for c in d['spec']['template']['spec']['containers']:
                    if any(any(k in v.get('name', '').lower() for k in _TRACE_KEYS) for v in c.get('env', [])):
                        out.append(d['metadata']['name'])
                        break
            if out:
                self.add_reasoning_step(observation=f"Found {len(out)} services with tracing instrumentation",
                                        conclusion="These services can be analyzed for distributed traces")
            else:
                self.add_reasoning_step(observation="No services with tracing instrumentation found",
                                        conclusion="Unable to analyze traces without instrumented services")
                self.add_finding(component="Tracing Configuration",
                                 issue="No services are instrumented for distributed tracing", severity="low",
                                 evidence="No tracing environment variables found in service configurations",
                                 recommendation="Add tracing instrumentation to your services for better observability")
            return out
        except Exception as e:
            self.add_reasoning_step(observation=f"Error checking for tracing instrumentation: {str(e)}",
                                    conclusion="Unable to determine which services are instrumented for tracing")
            return []

    def _simulated(self, s):  # ref :209-381 (canned findings, kept verbatim in meaning)
        n = len(s)
        self.add_reasoning_step(observation=f"Checking for high-latency traces in {n} services",
                                conclusion="Beginning latency analysis")
        self.add_finding(component=f"Service/{s[0]}", issue="High latency detected in service calls", severity="medium",
                         evidence="Trace analysis shows p95 latency above 500ms for HTTP GET operations",
                         recommendation="Optimize database queries, add caching, or scale the service horizontally")
        self.add_reasoning_step(observation=f"Detected high latency in {s[0]} service",
                                conclusion="Service performance may be affecting overall application responsiveness")
        if n >= 2:
            self.add_finding(component=f"Service/{s[0]}→{s[1]}", issue=f"Slow communication between {s[0]} and {s[1]}",
                             severity="medium",
                             evidence="Trace analysis shows high latency (>200ms) in calls from service_a to service_b",
                             recommendation="Investigate network issues, optimize the API between these services, or consider co-locating them")
            self.add_reasoning_step(observation=f"Detected slow communication between {s[0]} and {s[1]}",
                                    conclusion="Inter-service communication may be a bottleneck")
        self.add_reasoning_step(observation=f"Checking for error traces in {n} services",
                                conclusion="Beginning error path analysis")
        self.add_finding(component=f"Service/{s[0]}", issue="Error traces detected in service", severity="high",
                         evidence="5% of traces show HTTP 500 responses in the past hour",
                         recommendation="Check service logs for corresponding errors and fix the underlying issue")
        self.add_reasoning_step(observation=f"Detected error traces in {s[0]} service",
                                conclusion="Service is experiencing errors that may affect user experience")
        if n >= 3:
            self.add_finding(component=f"Services/{s[0]}→{s[1]}→{s[2]}", issue="Cascading failures detected in service chain",
                             severity="critical", evidence=f"Errors in {s[2]} are causing failures in {s[1]} and {s[0]}",
                             recommendation="Implement circuit breakers and fallback mechanisms to prevent cascading failures")
            self.add_reasoning_step(observation=f"Detected cascading failures from {s[2]} to {s[0]}",
                                    conclusion="Failure isolation mechanisms may be missing in the service architecture")
        self.add_reasoning_step(observation=f"Analyzing service dependencies among {n} services",
                                conclusion="Beginning dependency analysis")
        if n >= 2:
            b = s[n // 2]
            self.add_finding(component=f"Service/{s[0]}", issue=f"High dependency on {b}", severity="medium",
                             evidence=f"{s[0]} makes frequent calls to {b}, creating a tight coupling",
                             recommendation="Consider implementing caching, circuit breakers, or redesigning the interaction pattern")
            self.add_reasoning_step(observation=f"Detected high dependency of {s[0]} on {b}",
                                    conclusion="Service coupling may lead to reliability issues if the dependency fails")
        if n >= 3:
            self.add_finding(component=f"Services/{s[0]}↔{s[1]}↔{s[2]}", issue="Circular dependency detected between services",
                             severity="high",
                             evidence=f"Traces show a circular call pattern: {s[0]} → {s[1]} → {s[2]} → {s[0]}",
                             recommendation="Refactor the service architecture to remove circular dependencies")
            self.add_reasoning_step(observation=f"Detected circular dependency between {s[0]}, {s[1]}, and {s[2]}",
                                    conclusion="Circular dependencies may lead to deadlocks and complicate scaling")
