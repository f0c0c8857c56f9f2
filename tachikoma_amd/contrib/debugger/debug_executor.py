"""Debug executor with the reference's per-node dump layout
(python/tvm/contrib/debugger/debug_executor.py:37-347, debug_result.py:25-292).

    m = debug_executor.create(lib, tachikoma_amd.rocm(0), dump_root="/tmp/tkdbg")
    m.set_input("data", x)
    m.run()          # per-node timing + every node output dumped
    # /tmp/tkdbg/_tvmdbg_device_ROCM_0/{_tvmdbg_graph_dump.json, output_tensors.params,
    #                                   _tvmdbg_execution_trace.json}

Files, as the reference writes them:
  * ``_tvmdbg_graph_dump.json`` — the executor graph (``nodes``, ``arg_nodes``,
    ``node_row_ptr``, ``heads``, ``attrs`` with dltype/shape/storage_id), written at
    creation, nodes rewritten like DebugResult._update_graph_json (input names, ``op``,
    ``attrs.T``, ``shape``);
  * ``output_tensors.params`` — NDArray-list (file_utils.cc:210-236) of every node's output,
    keyed ``{name}____topo-index:{i}____output-num:{j}`` (debug_result.py:124), graph
    inputs and params included as ``param`` nodes;
  * ``_tvmdbg_execution_trace.json`` — Chrome trace, B/E events per node, pid = tid = 1,
    ``displayTimeUnit`` "ns" (debug_result.py:151-189).

Granularity (``create(..., granularity=)``):
  * ``"fused"`` (default, the reference's): one graph node per FuseOps-fused primitive
    function (relay/fuse.py: fuse_ops.cc partitioning, te_compiler_cache.cc naming, e.g.
    ``tvmgen_default_fused_qnn_conv2d_nn_bias_add_qnn_requantize_clip_3``); its output is the
    value of the group's last op, and params appear as ``null`` nodes before their first
    consumer, as the graph codegen emits bound constants;
  * ``"canonical"``: the fused functions of the graph the reference's executor actually runs --
    QNN legalized / canonicalized to int16 shifts, int16 contractions and the integer requantize
    chain, simplified (relay/canonical.py) -- so node names are the reference's own
    (``tvmgen_default_fused_nn_conv2d_add_fixed_point_multiply_per_axis_add_clip_cast``) and
    node values are the canonical tensors: plan records where one holds the value, the rest
    (int16 operand shifts, int32 partial sums) computed on the device (canonical_values.py);
  * ``"op"``: one graph node per Relay op (MRT names ``%N``), finer than the reference.
Device time of a node is the time of the device kernels that write its records (a device
block's time goes to the node holding its first op).
"""
from __future__ import annotations

import json
import os
import shutil
import tempfile
from typing import Dict, List, Optional

import numpy as np

from ... import trace_format as tf
from ..graph_executor import GraphModule

DUMP_ROOT_PREFIX = "tvmdbg_"
DUMP_PATH_PREFIX = "_tvmdbg_"
GRAPH_DUMP_FILE_NAME = "_tvmdbg_graph_dump.json"
CHROME_TRACE_FILE_NAME = "_tvmdbg_execution_trace.json"
OUTPUT_TENSORS_FILE_NAME = "output_tensors.params"


def executor_graph_json(plan, granularity: str = "op", mod_name: str = "default") -> dict:
    """The plan as a graph-executor JSON graph (graph_executor.h:226-340 layout).

    ``"op"``: null nodes for graph inputs and params, one tvm_op node per op, topological.
    ``"fused"``: null nodes for graph inputs, then the fused calls in the graph codegen's post
    order, each preceded by null nodes for the params it uses first
    (graph_executor_codegen.cc:408-472).  ``"outputs"`` maps every node to the plan tensor
    holding its value (the fused group's last op for a fused node)."""
    nodes: List[dict] = []
    index: Dict[str, int] = {}
    dltype: List[str] = []
    shapes: List[List[int]] = []
    outputs: List[str] = []
    arg_nodes: List[int] = []

    def null(t):
        index[t.name] = len(nodes)
        arg_nodes.append(len(nodes))
        nodes.append({"op": "null", "name": t.name, "inputs": []})
        dltype.append(t.dtype)
        shapes.append([int(d) for d in t.shape])
        outputs.append(t.name)

    def call(name, func_name, inputs, out):
        index[out.name] = len(nodes)
        nodes.append({"op": "tvm_op", "name": name, "inputs": [[index[x], 0, 0] for x in inputs],
                      "attrs": {"func_name": func_name, "num_inputs": str(len(inputs)), "num_outputs": "1",
                                "flatten_data": "0"}})
        dltype.append(out.dtype)
        shapes.append([int(d) for d in out.shape])
        outputs.append(out.name)

    if granularity == "op":
        for t in list(plan.inputs) + list(plan.params):
            null(t)
        for op in plan.ops:
            call(op.name, "tachikoma_" + op.op.replace(".", "_"), op.inputs, op.out)
    elif granularity in ("fused", "canonical"):
        from ...relay.fuse import fused_nodes
        if granularity == "canonical":
            from ...relay.canonical import canonicalize
            plan = canonicalize(plan)
        params = {t.name: t for t in plan.params}
        for t in plan.inputs:
            null(t)
        for fn in fused_nodes(plan, mod_name):
            for x in fn.inputs:
                if x in params and x not in index:
                    null(params[x])
            call(fn.node_name, fn.func_name, fn.inputs, fn.ops[-1].out)
    else:
        raise ValueError(f"granularity must be 'fused', 'canonical' or 'op', not {granularity!r}")
    return {
        "nodes": nodes,
        "arg_nodes": arg_nodes,
        "node_row_ptr": list(range(len(nodes) + 1)),
        "heads": [[index[o], 0, 0] for o in plan.outputs],
        "attrs": {"dltype": ["list_str", dltype], "shape": ["list_shape", shapes],
                  "storage_id": ["list_int", list(range(len(nodes)))]},
        "outputs": outputs,
    }


def _debug_nodes(graph: dict) -> List[dict]:
    """DebugResult._update_graph_json: input names, op = func_name or "param", attrs.T, shape."""
    nodes = json.loads(json.dumps(graph["nodes"]))
    dtypes = graph["attrs"]["dltype"][1]
    shapes = graph["attrs"]["shape"][1]
    for i, node in enumerate(nodes):
        node["inputs"] = [nodes[x[0]]["name"] for x in node["inputs"]]
        if "attrs" not in node:
            node["attrs"] = {}
            node["op"] = "param"
        else:
            node["op"] = node["attrs"]["func_name"]
        node["attrs"].update({"T": "type: " + dtypes[i]})
        node["shape"] = shapes[i]
    return nodes


class GraphModuleDebug(GraphModule):
    """GraphModule + the debug executor's dump (debug_executor.py:89-347)."""

    def __init__(self, module, device_name: str, dump_root: Optional[str] = None, granularity: str = "fused",
                 mod_name: str = "default"):
        super().__init__(module)
        self._dump_root = dump_root or tempfile.mkdtemp(prefix=DUMP_ROOT_PREFIX)
        folder = DUMP_PATH_PREFIX + "device_" + device_name.upper().replace("(", ":").replace(")", "").replace(":", "_")
        self._dump_path = os.path.join(self._dump_root, folder)
        os.makedirs(self._dump_path, 0o700, exist_ok=True)
        self.granularity = granularity
        self.mod_name = mod_name
        self.canon = None
        if granularity == "canonical":
            from ...relay.canonical import canonicalize
            self.canon = canonicalize(self.plan)
        graph = executor_graph_json(self.plan, granularity, mod_name)
        self._node_outputs: List[str] = graph.pop("outputs")
        self._graph = graph
        self._nodes = _debug_nodes(self._graph)
        with open(os.path.join(self._dump_path, GRAPH_DUMP_FILE_NAME), "w") as f:
            json.dump({**self._graph, "nodes": self._nodes}, f, indent=4, sort_keys=False)
        self._times_s: List[List[float]] = []
        self._outputs: Dict[int, np.ndarray] = {}

    @property
    def dump_path(self) -> str:
        return self._dump_path

    def _graph_node_of(self) -> List[Optional[int]]:
        """Graph node charged with each device node's time: the node holding its first record's
        op; a shadow node (no record) and a node whose records no graph node holds are charged to
        the next device node's graph node (None when no later one exists)."""
        node_of: Dict[str, int] = {}
        if self.granularity == "fused":
            from ...relay.fuse import fused_nodes
            op_nodes = [i for i, n in enumerate(self._nodes) if n["op"] != "param"]
            for gi, fn in zip(op_nodes, fused_nodes(self.plan, self.mod_name)):
                for op in fn.ops:
                    node_of[op.name] = gi
        elif self.granularity == "canonical":
            # a device node's time goes to the fused function holding the first canonical op
            # lowered from its first record's plan op
            from ...relay.fuse import fused_nodes
            op_nodes = [i for i, n in enumerate(self._nodes) if n["op"] != "param"]
            for gi, fn in zip(op_nodes, fused_nodes(self.canon, self.mod_name)):
                for op in fn.ops:
                    node_of.setdefault(op.origin, gi)
        else:
            for i, n in enumerate(self._nodes):
                node_of[n["name"]] = i
        direct = [next((node_of[r] for r in recs if r in node_of), None) for recs in self.module.node_records]
        out: List[Optional[int]] = [None] * len(direct)
        nxt = None
        for i in range(len(direct) - 1, -1, -1):  # carried nodes take the next charged node's
            if direct[i] is not None:
                nxt = direct[i]
            out[i] = nxt
        return out

    def _node_times(self, repeat: int) -> List[List[float]]:
        """Device seconds per graph node from whole-graph profiled runs (tk_module_run_profiled:
        HIP events around every device node of one run)."""
        owner = self._graph_node_of()
        per_node: List[List[float]] = [[] for _ in self._nodes]
        for _ in range(max(1, repeat)):
            times = list(self.module.run_profiled().values())  # ms per device node, in node order
            acc = [0.0] * len(self._nodes)
            for gi, ms in zip(owner, times):
                if gi is not None:
                    acc[gi] += ms * 1e-3
            for i, t in enumerate(acc):
                per_node[i].append(t)
        return per_node

    def _node_index(self, node) -> int:
        """debug_executor.py:252-276: a graph node index, or a node name (AttributeError when none
        has it)."""
        if isinstance(node, str):
            for i, n in enumerate(self._nodes):
                if n["name"] == node:
                    return i
            raise AttributeError(f"Could not find a node named {node} in this graph.")
        if isinstance(node, (int, np.integer)):
            if not 0 <= int(node) < len(self._nodes):
                raise IndexError(f"node index {node} out of range [0, {len(self._nodes)})")
            return int(node)
        raise RuntimeError("Require node index or name only.")

    def debug_get_output(self, node, out=None):
        """debug_executor.py:252-276 (GraphExecutorDebug::DebugGetNodeOutput): run the graph and
        return graph node ``node``'s value (an index or a name); copied into ``out`` (a numpy
        array) when given.  Every node's value is kept in its own device buffer, so the whole graph
        runs and the node's buffer is read -- the value the reference computes by running up to
        the node."""
        i = self._node_index(node)
        GraphModule.run(self)
        if self.canon is not None:
            from .canonical_values import CanonicalValues
            t = CanonicalValues(self.module, self.canon).value(self._node_outputs[i])
        else:
            t = self.module.buffers[self._node_outputs[i]]
        if out is not None:
            out[...] = t.detach().cpu().numpy()
            return out
        from ..graph_executor import NDArrayView
        return NDArrayView(t)

    def run_individual_node(self, index: int, number: int = 10, repeat: int = 1, min_repeat_ms: int = 0,
                            limit_zero_time_iterations: int = 100, cooldown_interval_ms: int = 0,
                            repeats_to_cooldown: int = 1):
        """debug_executor.py:415-480 (GraphExecutorDebug::RunIndividualNode,
        graph_executor_debug.cc:118-144): time graph node ``index`` alone on data already on the
        device -- its device nodes (and the shadow nodes charged to it) re-run back to back,
        ``number`` times per measurement, ``repeat`` measurements, HIP-event timed on the current
        stream.  A param / input node runs nothing: ``repeat`` zeros.  Returns a BenchmarkResult
        of seconds per run."""
        from ..graph_executor import BenchmarkResult, time_evaluator
        i = self._node_index(index)
        owner = self._graph_node_of()
        mine = [k for k, gi in enumerate(owner) if gi == i]
        if not mine:
            return BenchmarkResult([0.0] * max(1, repeat))
        spans: List[List[int]] = []
        for k in mine:  # consecutive device nodes -> one tk_module_run_range
            if spans and spans[-1][1] == k:
                spans[-1][1] = k + 1
            else:
                spans.append([k, k + 1])
        import torch
        stream = torch.cuda.current_stream(self.module.device)

        def call():
            for b, e in spans:
                self.module.run_range(b, e, stream)
        return BenchmarkResult(time_evaluator(call, self.module.device, number, repeat, min_repeat_ms,
                                              limit_zero_time_iterations, cooldown_interval_ms, repeats_to_cooldown))

    def run_individual(self, number: int, repeat: int = 1, min_repeat_ms: int = 0,
                       limit_zero_time_iterations: int = 100, cooldown_interval_ms: int = 0,
                       repeats_to_cooldown: int = 1) -> List[List[float]]:
        """debug_executor.py:349-413 (GraphExecutorDebug::RunIndividual, graph_executor_debug.cc:
        70-116): one warm-up run of the graph, then every graph node timed alone
        (run_individual_node); a list with one entry per graph node -- ``repeat`` seconds-per-run
        values each, zeros for param / input nodes."""
        GraphModule.run(self)
        return [self.run_individual_node(i, number, repeat, min_repeat_ms, limit_zero_time_iterations,
                                         cooldown_interval_ms, repeats_to_cooldown).results
                for i in range(len(self._nodes))]

    def profile(self, collectors=None, **input_dict) -> "Report":
        """debug_executor.py:482-503 (GraphExecutorDebug::Profile): run the graph once and report
        per-call device time (one call per executed graph node, in execution order) and the
        whole-graph time.  ``collectors`` (hardware metric collectors) are not supported: pass
        None; rocprofv3 counters are this engine's collectors (tools/pmc.sh)."""
        if collectors:
            raise NotImplementedError("profile(collectors=...): use rocprofv3 --pmc (tools/pmc.sh)")
        if input_dict:
            self.set_input(**input_dict)
        times = self._node_times(1)
        calls = []
        for node, t in zip(self._nodes, times):
            if node["op"] == "param":
                continue
            calls.append({"Name": node["name"], "Duration (us)": t[0] * 1e6, "Count": 1,
                          "Device": f"rocm{self.module.device.index or 0}", "Hash": node["op"],
                          "Argument Shapes": str(tuple(node["shape"]))})
        total = sum(c["Duration (us)"] for c in calls)
        for c in calls:
            c["Percent"] = c["Duration (us)"] / total * 100 if total else 0.0
        return Report(calls, {"Executor": "GraphModuleDebug", "Granularity": self.granularity,
                              "Duration (us)": total})

    def run(self, repeat: int = 1, sort_by_time: bool = True, **inputs):  # noqa: D401  (debug_executor.run)
        """Execute, time every node, dump the output tensors and the Chrome trace, print the table."""
        if inputs:
            self.set_input(**inputs)
        self._times_s = self._node_times(repeat)
        if self.canon is not None:
            from .canonical_values import CanonicalValues
            vals = CanonicalValues(self.module, self.canon)
            dev = [vals.value(name) for name in self._node_outputs]
            self._outputs = {i: t.detach().cpu().numpy() for i, t in enumerate(dev)}
        else:
            self._outputs = {i: self.module.buffers[name].detach().cpu().numpy()
                             for i, name in enumerate(self._node_outputs)}
        self.dump_output_tensor()
        self.dump_chrome_trace()
        self.display_debug_result(sort_by_time)

    def get_output_tensors(self) -> Dict[str, np.ndarray]:
        """debug_result.py:114-127: keyed ``{name}____topo-index:{i}____output-num:{j}``."""
        return {f"{n['name']}____topo-index:{i}____output-num:0": self._outputs[i]
                for i, n in enumerate(self._nodes)}

    def node_outputs(self) -> List[str]:
        """Plan tensor holding each graph node's value (a fused node: its group's last op; with
        granularity "canonical", the canonical tensor)."""
        return list(self._node_outputs)

    def dump_output_tensor(self) -> None:
        with open(os.path.join(self._dump_path, OUTPUT_TENSORS_FILE_NAME), "wb") as f:
            f.write(tf.save_ndarray_list(self.get_output_tensors()))

    def dump_chrome_trace(self) -> None:
        starts = np.zeros(len(self._times_s) + 1)
        starts[1:] = np.cumsum([np.mean(t) for t in self._times_s])
        events = []
        for node, times, t0 in zip(self._nodes, self._times_s, starts):
            events.append({"ts": t0 * 1e6, "tid": 1, "pid": 1, "name": node["name"], "ph": "B"})
            events.append({"ts": (np.mean(times) + t0) * 1e6, "tid": 1, "pid": 1, "name": node["name"], "ph": "E"})
        with open(os.path.join(self._dump_path, CHROME_TRACE_FILE_NAME), "w") as f:
            json.dump({"displayTimeUnit": "ns", "traceEvents": events}, f)

    def get_debug_result(self, sort_by_time: bool = True) -> str:
        header = ["Node Name", "Ops", "Time(us)", "Time(%)", "Shape", "Inputs", "Outputs", "Measurements(us)"]
        lines = ["---------", "---", "--------", "-------", "-----", "------", "-------", "----------------"]
        total = sum(float(np.mean(t)) for t in self._times_s)
        data = []
        for node, times in zip(self._nodes, self._times_s):
            if node["op"] == "param":
                continue
            mean = float(np.mean(times))
            data.append([node["name"], node["op"], round(mean * 1e6, 3),
                         round(mean / total * 100, 3) if total else 0.0, str(tuple(node["shape"])),
                         node["attrs"]["num_inputs"], node["attrs"]["num_outputs"],
                         str([round(t * 1e6, 3) for t in times])])
        if sort_by_time:
            data = sorted(data, key=lambda r: r[2], reverse=True)
            data.append(["Total_time", "-", round(total * 1e6, 3), "-", "-", "-", "-", "-", "-"])
        widths = [max(len(header[i]), *(len(str(r[i])) for r in data)) + 2 for i in range(len(header))]
        fmt = "".join("{:<" + str(w) + "}" for w in widths)
        out = [fmt.format(*header), fmt.format(*lines)]
        out += [fmt.format(*r[:len(header)]) for r in data]
        return "\n".join(out)

    def display_debug_result(self, sort_by_time: bool = True) -> None:
        print(self.get_debug_result(sort_by_time))

    def exit(self) -> None:
        """Remove the dump root (debug_executor.py:505-510)."""
        if os.path.isdir(self._dump_root):
            shutil.rmtree(self._dump_root)


class Report:
    """What profile() returns (python/tvm/runtime/profiling/__init__.py Report): ``calls`` (one
    dict per call: Name, Duration (us), Percent, Count, Device, Hash, Argument Shapes) and
    ``configuration``; ``table()`` / ``csv()`` / ``json()`` renderings."""

    COLUMNS = ("Name", "Duration (us)", "Percent", "Count", "Device", "Argument Shapes")

    def __init__(self, calls: List[dict], configuration: dict):
        self.calls = calls
        self.configuration = configuration

    def table(self, sort: bool = True, aggregate: bool = True, col_sums: bool = True) -> str:
        rows = list(self.calls)
        if aggregate:
            agg: Dict[str, dict] = {}
            for c in rows:
                a = agg.setdefault(c["Name"], dict(c, **{"Duration (us)": 0.0, "Percent": 0.0, "Count": 0}))
                a["Duration (us)"] += c["Duration (us)"]
                a["Percent"] += c["Percent"]
                a["Count"] += c["Count"]
            rows = list(agg.values())
        if sort:
            rows.sort(key=lambda c: -c["Duration (us)"])
        if col_sums:
            rows.append({"Name": "Sum", "Duration (us)": sum(c["Duration (us)"] for c in rows),
                         "Percent": sum(c["Percent"] for c in rows), "Count": sum(c["Count"] for c in rows),
                         "Device": "", "Argument Shapes": ""})
        cells = [[f"{c[k]:.2f}" if isinstance(c[k], float) else str(c[k]) for k in self.COLUMNS] for c in rows]
        widths = [max(len(h), *(len(r[i]) for r in cells)) for i, h in enumerate(self.COLUMNS)] if cells else \
            [len(h) for h in self.COLUMNS]
        lines = ["  ".join(h.ljust(w) for h, w in zip(self.COLUMNS, widths))]
        lines += ["  ".join(v.ljust(w) for v, w in zip(r, widths)) for r in cells]
        lines.append("Configuration")
        lines.append("-------------")
        lines += [f"{k}: {v}" for k, v in self.configuration.items()]
        return "\n".join(lines)

    def csv(self) -> str:
        out = [",".join(f'"{h}"' for h in self.COLUMNS)]
        out += [",".join(f'"{c[k]}"' for k in self.COLUMNS) for c in self.calls]
        return "\n".join(out)

    def json(self) -> str:
        return json.dumps({"calls": self.calls, "configuration": self.configuration})

    def __str__(self) -> str:
        return self.table()


def create(lib_factory, dev=None, dump_root: Optional[str] = None, granularity: str = "fused") -> GraphModuleDebug:
    """``debug_executor.create`` analogue taking what ``relay.build`` returns."""
    module = lib_factory[lib_factory.mod_name](dev)
    dev_id = int(module.device.index or 0)
    return GraphModuleDebug(module, f"rocm({dev_id})", dump_root, granularity, lib_factory.mod_name)
