"""LogsAgent: per-container 13-category line histograms on the device.

Reference: ref:agents/logs_agent.py:4-477.  The hot loop is ``_analyze_container_logs``
(:124-181): ``logs.splitlines()`` then, for each of 13 regexes, the lines that
``re.search(p, line, re.IGNORECASE)``.  Here every container's log text is packed into one
UTF-8 blob (``doc_off`` = byte offset of each container's text) and ``krca_log_scan`` splits
lines, runs the compiled DFA (csrc/log_dfa_tables.h) and builds, atomics-free, the per-container
line count, 13-bin histogram and the first three matching lines per bin.  The host only turns
those into the reference's findings (same order, strings, evidence truncation).

Container status, pod conditions, init containers and the "no logs" check (:183-414) are
dict walks and stay on the host with the reference's semantics — including its bugs, which
parity depends on (SURVEY.md §7 "Reference bugs that parity must preserve").
"""
import numpy as np

from .base import BaseAgent
from .. import patterns as P


def pack_documents(texts):
    """list[str] -> (utf-8 blob bytes, int64 doc_off[D+1]).  Lone surrogates pass through."""
    enc = [t.encode("utf-8", "surrogatepass") for t in texts]
    off = np.zeros(len(enc) + 1, dtype=np.int64)
    if enc:
        off[1:] = np.cumsum([len(e) for e in enc])
    return b"".join(enc), off


def format_examples(lines, n):
    """Evidence text of ref:agents/logs_agent.py:159-163."""
    text = "\n".join(f"- {ln[:200]}..." if len(ln) > 200 else f"- {ln}" for ln in lines[:3])
    if n > 3:
        text += f"\n- ... and {n - 3} more similar errors"
    return text


class LogsAgent(BaseAgent):
    def __init__(self, k8s_client, engine=None):
        super().__init__(k8s_client, engine)
        self.error_patterns = dict(P.ERROR_PATTERNS)  # public attribute of the reference (:20)

    def _check_patterns_compiled(self):
        """The device matcher is compiled from krca/patterns.py (csrc/gen_log_dfa.py); the reference
        matches whatever self.error_patterns holds (ref:agents/logs_agent.py:20,147-149).  An edited
        dict would silently give different histograms, so it is refused instead."""
        ident = getattr(self.engine, "log_dfa_identity", None)
        if ident is not None and ident()[1] != P.pattern_digest():
            raise P.PatternsChanged("krca/patterns.py and the compiled matcher (libkrca.so) disagree: "
                                    "regenerate csrc/log_dfa_tables.h and rebuild")
        if list(self.error_patterns.items()) == list(P.ERROR_PATTERNS):
            return
        raise P.PatternsChanged(
            "LogsAgent.error_patterns differs from the patterns the device matcher was compiled from "
            "(krca/patterns.py); edit krca/patterns.py and regenerate csrc/log_dfa_tables.h with "
            "csrc/gen_log_dfa.py")

    def analyze(self, namespace, context=None, **kwargs):
        self.reset()
        try:
            self._maybe_set_context(context)
            pods = self.k8s_client.get_pods(namespace)
            if not pods:
                self.add_reasoning_step(observation=f"No pods found in namespace {namespace}",
                                        conclusion="Unable to analyze logs as no pods were found")
                return self.get_results()
            self.add_reasoning_step(observation=f"Found {len(pods)} pods in namespace {namespace}",
                                    conclusion="Beginning logs analysis for each pod")
            terminated = self.k8s_client.get_recently_terminated_pods(namespace)
            if terminated:
                self.add_reasoning_step(observation=f"Found {len(terminated)} recently terminated pods",
                                        conclusion="Will analyze logs from terminated pods as well")
                pods.extend(terminated)

            # (1) gather every container's text; a failure mid-way is re-raised only after the
            #     containers fetched before it are reported, exactly as the reference's loop does
            docs, deferred = [], None
            try:
                for pod in pods:
                    pod_name = pod["metadata"]["name"]
                    for container in pod["spec"]["containers"]:
                        cname = container["name"]
                        logs = self.k8s_client.get_pod_logs(pod_name, namespace, cname)
                        if logs:
                            docs.append((pod, pod_name, cname, logs))
            except Exception as e:  # noqa: BLE001 - re-raised below
                deferred = e

            # (2) one device pass over all containers
            if docs:
                self._check_patterns_compiled()
            scan = self.engine.log_scan(*pack_documents([d[3] for d in docs])) if docs else None

            # (3) findings in the reference's order: per container, log findings then status
            for i, (pod, pod_name, cname, logs) in enumerate(docs):
                self._report_container(scan, i, pod_name, cname)
                self._check_container_status(pod, cname)
            if deferred is not None:
                raise deferred

            self._analyze_pod_conditions(pods)
            self._analyze_init_containers(pods)
            self._check_for_no_logs(pods)
            return self.get_results()
        except Exception as e:  # ref:agents/logs_agent.py:113-122
            return self._error_result("logs", e)

    # -- ref:agents/logs_agent.py:124-181 on device results -------------------------------
    def _report_container(self, scan, d, pod_name, cname):
        n_lines = int(scan.n_lines[d])
        self.add_reasoning_step(observation=f"Analyzing {n_lines} log lines for {pod_name}/{cname}",
                                conclusion="Beginning log pattern analysis")
        hist = scan.hist[d]
        if not hist.any():
            self.add_reasoning_step(observation=f"No error patterns detected in logs for {pod_name}/{cname}",
                                    conclusion="Container logs appear normal")
            return
        for c, cat in enumerate(P.CATEGORY_NAMES):
            n = int(hist[c])
            if n == 0:
                continue
            ttl = P.title(cat)
            self.add_finding(component=f"Pod/{pod_name}/{cname}",
                             issue=f"Detected {n} instances of {ttl} in logs",
                             severity=P.severity(cat),
                             evidence=f"Log entries:\n{format_examples(scan.examples(d, c), n)}",
                             recommendation=P.recommendation(cat))
            self.add_reasoning_step(
                observation=f"Found {n} log entries matching {cat} pattern in {pod_name}/{cname}",
                conclusion=f"Container is experiencing {ttl} issues")

    # -- ref:agents/logs_agent.py:183-257 ------------------------------------------------
    def _check_container_status(self, pod, container_name):
        issues = []
        statuses = pod["status"].get("containerStatuses", []) + pod["status"].get("initContainerStatuses", [])
        st = next((s for s in statuses if s["name"] == container_name), None)
        if not st:
            return issues
        pod_name = pod["metadata"]["name"]
        comp = f"Pod/{pod_name}/{container_name}"
        restarts = st.get("restartCount", 0)
        if restarts > 5:
            issues.append(f"High restart count ({restarts})")
            self.add_finding(component=comp, issue=f"Container has restarted {restarts} times",
                             severity="high" if restarts > 10 else "medium",
                             evidence=f"Container {container_name} in pod {pod_name} has a restart count of {restarts}",
                             recommendation="Investigate logs for crash causes and ensure the container is properly configured")
        if not st.get("ready", True):
            last = st.get("lastState", {})
            if "terminated" in last:
                term = last["terminated"]
                code = term.get("exitCode", 0)
                reason = term.get("reason", "Unknown")
                if code != 0:
                    issues.append(f"Container terminated with exit code {code} ({reason})")
                    self.add_finding(component=comp, issue=f"Container terminated with non-zero exit code {code}",
                                     severity="high", evidence=f"Termination reason: {reason}",
                                     recommendation="Check container logs for error details and fix the underlying issue")
            elif "waiting" in last:
                w = last["waiting"]
                reason = w.get("reason", "Unknown")
                issues.append(f"Container in waiting state: {reason}")
                self.add_finding(component=comp, issue=f"Container is in waiting state with reason: {reason}",
                                 severity="medium", evidence=f"Waiting message: {w.get('message', '')}",
                                 recommendation="Address the issue preventing the container from starting")
        return issues

    # -- ref:agents/logs_agent.py:259-310 ------------------------------------------------
    def _analyze_pod_conditions(self, pods):
        n_issues = 0
        for pod in pods:
            pod_name = pod["metadata"]["name"]
            for cond in pod["status"].get("conditions", []):
                ctype, status = cond.get("type", ""), cond.get("status", "")
                reason, message = cond.get("reason", ""), cond.get("message", "")
                if ctype == "PodScheduled" and status == "False":
                    n_issues += 1
                    self.add_finding(component=f"Pod/{pod_name}", issue="Pod cannot be scheduled", severity="high",
                                     evidence=f"Reason: {reason}, Message: {message}",
                                     recommendation="Check node resources, taints, tolerations, and node selectors")
                elif ctype == "Ready" and status == "False":
                    n_issues += 1
                    self.add_finding(component=f"Pod/{pod_name}", issue="Pod is not in Ready state", severity="medium",
                                     evidence=f"Reason: {reason}, Message: {message}",
                                     recommendation="Investigate container statuses and logs for errors")
        if n_issues:
            self.add_reasoning_step(observation=f"Found {n_issues} pods with condition issues",
                                    conclusion="Pod conditions indicate scheduling or readiness problems")
        else:
            self.add_reasoning_step(observation="No pod condition issues detected",
                                    conclusion="All pods appear to be properly scheduled and ready")

    # -- ref:agents/logs_agent.py:312-372 ------------------------------------------------
    def _analyze_init_containers(self, pods):
        n_issues = 0
        for pod in pods:
            pod_name = pod["metadata"]["name"]
            for st in pod["status"].get("initContainerStatuses", []):
                cname = st.get("name", "")
                if st.get("ready", False):
                    continue
                state = st.get("state", {})
                comp = f"Pod/{pod_name}/init/{cname}"
                if "waiting" in state:
                    w = state["waiting"]
                    n_issues += 1
                    self.add_finding(component=comp,
                                     issue=f"Init container is waiting with reason: {w.get('reason', 'Unknown')}",
                                     severity="high", evidence=f"Message: {w.get('message', '')}",
                                     recommendation="Check init container logs and configuration")
                elif "terminated" in state:
                    t = state["terminated"]
                    code = t.get("exitCode", 0)
                    if code != 0:
                        n_issues += 1
                        self.add_finding(component=comp,
                                         issue=f"Init container terminated with non-zero exit code {code}",
                                         severity="high", evidence=f"Termination reason: {t.get('reason', 'Unknown')}",
                                         recommendation="Check init container logs for error details")
        if n_issues:
            self.add_reasoning_step(observation=f"Found {n_issues} init container issues",
                                    conclusion="Init container failures are preventing pods from starting")
        else:
            self.add_reasoning_step(observation="No init container issues detected",
                                    conclusion="All init containers appear to be functioning correctly")

    # -- ref:agents/logs_agent.py:374-414 (keeps the str - str TypeError of :402) ---------
    def _check_for_no_logs(self, pods):
        for pod in pods:
            if pod["status"].get("phase", "") != "Running":
                continue
            pod_name = pod["metadata"]["name"]
            for container in pod["spec"]["containers"]:
                cname = container["name"]
                logs = self.k8s_client.get_pod_logs(pod_name, pod["metadata"]["namespace"], cname)
                if logs:
                    continue
                start_time = pod["status"].get("startTime", "")
                current_time = self.k8s_client.get_current_time()
                if start_time and (current_time - start_time).total_seconds() > 300:
                    self.add_finding(component=f"Pod/{pod_name}/{cname}",
                                     issue="Container has been running for over 5 minutes but has no logs",
                                     severity="medium",
                                     evidence=f"No log output detected for container {cname}",
                                     recommendation="Verify the application is properly writing to stdout/stderr and not failing silently")
                    self.add_reasoning_step(
                        observation=f"No logs found for {pod_name}/{cname} despite running state",
                        conclusion="Container may be failing silently or not properly logging to stdout/stderr")

    # public helpers of the reference kept for API compatibility
    def _determine_error_severity(self, error_type):
        return P.severity(error_type)

    def _format_error_type(self, error_type):
        return P.title(error_type)

    def _get_recommendation_for_error(self, error_type):
        return P.recommendation(error_type)
