"""Coordinator: dispatch, cross-agent correlation, root causes (+ device PageRank ranking).

Reference: ref:agents/coordinator.py:7-192.  ``run_analysis`` / the comprehensive result
schema / ``_correlate_findings`` (group by component, first-seen order, max severity by
:data:`SEVERITY_ORDER`) / ``_identify_root_causes`` (critical|high with >1 finding) are kept
exactly.  New, additive: ``ranked_root_causes`` — the root-cause ranking
of krca.rca.Config (the same definition bench.py and RcaStep use: alpha 0.5, p ∝ max(s - floor, 0)
with the scale-aware floor of Config.floor -- the expected maximum |z| of that many null series,
at least 4 -- 30 iterations, key "explained": the mass a pod received from its callers times the
part of its anomaly no anomalous dependency explains) over the dependency graph, seeded by the metrics agent's anomaly scores
(bulk path) or by the trace backend's per-service error rates (C1 mock; error rates are not in
|z| units, so that path seeds with floor 0), computed by ``krca_ppr`` on the device.
"""
import numpy as np

from .base import SEVERITY_ORDER
from .events import EventsAgent
from .logs import LogsAgent
from .metrics import MetricsAgent
from .topology import TopologyAgent, csr_from_edges
from .traces import TracesAgent


class Coordinator:
    def __init__(self, k8s_client, engine=None, rank_config=None):
        from krca.rca import RANKING
        self.k8s_client = k8s_client
        self._engine = engine
        self.rank_config = rank_config or RANKING
        self.metrics_agent = MetricsAgent(k8s_client, engine, window=self.rank_config.window,
                                          z_threshold=self.rank_config.z_threshold)
        self.logs_agent = LogsAgent(k8s_client, engine)
        self.traces_agent = TracesAgent(k8s_client, engine)
        self.topology_agent = TopologyAgent(k8s_client, engine)
        self.events_agent = EventsAgent(k8s_client, engine)
        self.agent_map = {
            'comprehensive': self._run_comprehensive_analysis,
            'metrics': self.metrics_agent.analyze,
            'logs': self.logs_agent.analyze,
            'traces': self.traces_agent.analyze,
            'topology': self.topology_agent.analyze,
            'events': self.events_agent.analyze,
        }

    @property
    def engine(self):
        if self._engine is None:
            from krca import native
            self._engine = native.default_engine()
        return self._engine

    def run_analysis(self, analysis_type, namespace, context=None, **kwargs):  # ref :39-70
        try:
            if analysis_type not in self.agent_map:
                return {'error': f"Unknown analysis type: {analysis_type}"}
            results = self.agent_map[analysis_type](namespace=namespace, context=context, **kwargs)
            results['metadata'] = {'analysis_type': analysis_type, 'namespace': namespace,
                                   'context': context or self.k8s_client.get_current_context(),
                                   'timestamp': self.k8s_client.get_current_time()}
            return results
        except Exception as e:
            return {'error': str(e)}

    def _run_comprehensive_analysis(self, namespace, context=None, **kwargs):  # ref :72-116
        self._reset_agents()
        order = ('metrics', 'logs', 'topology', 'events', 'traces')
        agents = {'metrics': self.metrics_agent, 'logs': self.logs_agent, 'topology': self.topology_agent,
                  'events': self.events_agent, 'traces': self.traces_agent}
        results = {k: agents[k].analyze(namespace, context, **kwargs) for k in order}
        correlated = self._correlate_findings(*(results[k].get('findings', []) for k in order))
        out = {'correlated_findings': correlated, 'agent_results': results,
               'root_causes': self._identify_root_causes(correlated)}
        ranked = self._rank_root_causes(namespace)
        if ranked is not None:
            out['ranked_root_causes'] = ranked
        return out

    def _correlate_findings(self, *lists):  # ref :118-155
        """Group by component (first-seen order), keep groups with > 1 finding, max severity by
        SEVERITY_ORDER.  The group-by runs on the device (krca_group_reduce, f4): component ids
        interned here, severity index as the key; member lists are split on the host."""
        flat = [f for lst in lists for f in lst]
        if not flat:
            return []
        ids, comps = {}, []
        slot = np.empty(len(flat), np.int32)
        sev = np.empty(len(flat), np.int64)
        for i, f in enumerate(flat):
            c = f['component']
            slot[i] = j = ids.setdefault(c, len(ids))
            if j == len(comps):
                comps.append(c)
            s = f['severity']
            sev[i] = SEVERITY_ORDER.index(s) if type(s) is str and s in SEVERITY_ORDER else -1
        S = len(comps)
        first, count, n_key, top = self.engine.group_reduce(slot, sev, S, 1)
        order = np.argsort(slot, kind='stable')
        members = np.split(order, np.cumsum(count)[:-1])
        out = []
        for g in np.argsort(first, kind='stable').tolist():
            if count[g] < 2:
                continue
            if n_key[g] != count[g]:  # the reference's max(key=list.index) raises on the first bad one
                for i in members[g].tolist():
                    list(SEVERITY_ORDER).index(flat[i]['severity'])
            out.append({'component': comps[g], 'related_findings': [flat[i] for i in members[g].tolist()],
                        'correlation_type': 'component', 'severity': SEVERITY_ORDER[int(top[0, g])]})
        return out

    @staticmethod
    def _identify_root_causes(correlated):  # ref :157-184
        out = []
        for c in correlated:
            n = len(c['related_findings'])
            if c['severity'] in ('critical', 'high') and n > 1:
                out.append({'component': c['component'], 'related_findings_count': n, 'severity': c['severity'],
                            'explanation': f"High severity issue with {n} related findings indicates a potential root cause."})
        return out

    def _reset_agents(self):
        for a in (self.metrics_agent, self.logs_agent, self.traces_agent, self.topology_agent, self.events_agent):
            a.reset()

    # -- additive ranking ----------------------------------------------------------------
    def _rank_root_causes(self, namespace):
        c = self.k8s_client
        scores = self.metrics_agent.last_scores
        if scores is not None and hasattr(c, 'get_dependency_csr'):
            names, row_ptr, col, outdeg = c.get_dependency_csr(namespace)
            zl = scores.get('z_last')
            idx, val, rank = self.engine.rank_root_causes(scores['score'], row_ptr, col, outdeg, self.rank_config,
                                                          n_metrics=int(zl.shape[1]) if zl is not None else 1)
            sc = np.asarray(scores['score'].cpu() if hasattr(scores['score'], 'cpu') else scores['score'])
            return [{'component': f"Pod/{names[i]}", 'rank': r + 1, 'score': float(v), 'pagerank': float(rank[i]),
                     'anomaly': float(sc[i])} for r, (i, v) in enumerate(zip(idx.tolist(), val.tolist()))]
        if hasattr(c, 'get_service_dependencies') and hasattr(c, 'get_error_rate_by_service'):
            deps = c.get_service_dependencies()
            rates = c.get_error_rate_by_service()
            names = list(deps.keys())
            for ds in deps.values():
                for d in ds:
                    if d not in names:
                        names.append(d)
            pos = {n: i for i, n in enumerate(names)}
            src = [pos[s] for s, ds in deps.items() for _ in ds]
            dst = [pos[d] for _, ds in deps.items() for d in ds]
            row_ptr, col, outdeg = csr_from_edges(len(names), src, dst)
            seed = np.array([rates.get(n, 0.0) for n in names], dtype=np.float32)
            if not seed.sum() > 0:
                return None
            idx, val, rank = self.engine.rank_root_causes(seed, row_ptr, col, outdeg,
                                                          self.rank_config.replace(seed_floor=0.0))
            return [{'component': f"Service/{names[i]}", 'rank': r + 1, 'score': float(v), 'pagerank': float(rank[i]),
                     'anomaly': float(seed[i])} for r, (i, v) in enumerate(zip(idx.tolist(), val.tolist()))]
        return None
