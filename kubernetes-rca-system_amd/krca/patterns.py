"""The 13 ordered log error categories.

Data of ref:agents/logs_agent.py:20-34 (regexes, matched with ``re.IGNORECASE`` per line of
``logs.splitlines()``), :416-437 (severity), :439-449 (title), :451-477 (recommendation).
The regexes are compiled once, offline, into the device DFA tables in
``csrc/log_dfa_tables.h`` by ``csrc/gen_log_dfa.py``; Python never matches them on the
product path.
"""

ERROR_PATTERNS = (
    ("oom_kill", r"(Out of memory|OOMKilled|Killed|signal: killed)"),
    ("connection_refused", r"(Connection refused|connect: connection refused)"),
    ("permission_denied", r"(Permission denied|Forbidden|Access denied)"),
    ("timeout", r"(timeout|Timeout|timed out|ETIMEDOUT)"),
    ("crash_loop", r"(CrashLoopBackOff|Back-off restarting)"),
    ("api_error", r"(API server error|StatusCode=5\d\d)"),
    ("volume_mount", r"(Unable to mount volumes|MountVolume.SetUp failed)"),
    ("image_pull", r"(ErrImagePull|ImagePullBackOff)"),
    ("dns_resolution", r"(DNS resolution failed|could not resolve)"),
    ("authentication", r"(Unauthorized|Authentication failed)"),
    ("config_error", r"(Invalid configuration|ConfigMap not found|Secret not found)"),
    ("internal_server_error", r"(internal server error|InternalServerError|500 Internal Server Error)"),
    ("exception", r"(Exception|Error|Traceback|FATAL|CRITICAL|Panic|panic:)"),
)
N_CATEGORIES = len(ERROR_PATTERNS)
CATEGORY_NAMES = tuple(k for k, _ in ERROR_PATTERNS)

_HIGH = ("oom_kill", "crash_loop", "image_pull")
_MEDIUM = ("connection_refused", "timeout", "volume_mount", "dns_resolution", "internal_server_error")
_LOW = ("permission_denied", "authentication", "config_error")


def severity(category):
    if category in _HIGH:
        return "high"
    if category in _MEDIUM:
        return "medium"
    if category in _LOW:
        return "low"
    return "info"


def title(category):
    return " ".join(w.capitalize() for w in category.split("_"))


RECOMMENDATIONS = {
    "oom_kill": "Increase memory limits for the container or optimize the application's memory usage",
    "connection_refused": "Check network policies, service endpoints, and ensure the target service is running",
    "permission_denied": "Verify RBAC permissions, service account settings, and security contexts",
    "timeout": "Check for network issues, increase timeout values, or optimize the slow operation",
    "crash_loop": "Investigate container logs for crash causes and fix the underlying application issue",
    "api_error": "Check for Kubernetes API server issues or problems with the client configuration",
    "volume_mount": "Verify PVC status, storage class availability, and volume permissions",
    "image_pull": "Ensure the image exists, credentials are correct, and network connectivity to the registry",
    "dns_resolution": "Check CoreDNS/kube-dns functionality and network policies that might block DNS",
    "authentication": "Verify credentials, tokens, and authentication configuration",
    "config_error": "Check that all required ConfigMaps and Secrets exist and are correctly referenced",
    "internal_server_error": "Investigate server-side issues in the dependent service",
    "exception": "Debug the application code to fix the exception",
}


def recommendation(category):
    return RECOMMENDATIONS.get(category, "Investigate the logs in detail to identify the root cause")


class PatternsChanged(ValueError):
    """LogsAgent.error_patterns no longer matches the compiled device matcher."""


def pattern_digest(patterns=ERROR_PATTERNS):
    """FNV-1a 64 over the (name, pattern) pairs in order, NUL-separated: the identity of a
    compiled pattern set (KRCA_DFA_DIGEST in csrc/log_dfa_tables.h, krca_log_dfa_digest())."""
    h = 0xcbf29ce484222325
    for name, pat in patterns:
        for c in name.encode() + b"\0" + pat.encode() + b"\0":
            h = ((h ^ c) * 0x100000001b3) & 0xFFFFFFFFFFFFFFFF
    return h
