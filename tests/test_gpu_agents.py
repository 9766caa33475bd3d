"""The drop-in agents on the device path (libkrca) against the reference goldens."""
import pytest

import agent_cases as A
from krca import native

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    return native.NativeEngine()


def test_c1_raw(eng):
    assert A.check_c1(eng, "c1_raw.json", A.MockK8sClient) == []


def test_c1_shim(eng):
    assert A.check_c1(eng, "c1_shim.json", A.Shim) == []


def test_c1_other(eng):
    assert A.check_c1_other(eng) == []


def test_logs_corpus(eng):
    assert A.check_logs_corpus(eng) == []


def test_metrics_scaled(eng):
    assert A.check_metrics_scaled(eng) == []


def test_topology(eng):
    assert A.check_topology(eng) == []


def test_ranked_root_causes_c1(eng):
    res = A.Coordinator(A.Shim(), engine=eng).run_analysis("comprehensive", A.NS)
    assert [r["component"] for r in res["ranked_root_causes"]] == [
        "Service/database", "Service/backend", "Service/api-gateway", "Service/resource-service", "Service/frontend"]


def test_default_engine_is_native():
    e = native.default_engine()
    assert isinstance(e, native.NativeEngine)
    assert e.lib.krca_version() == 100
