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

    def _node_times(self, repeat: int) -> List[List[float]]:
        """Device seconds per graph node: each device node's time goes to the graph node that
        holds its first record's op (a shadow node's to the next device node's)."""
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
        per_node: List[List[float]] = [[] for _ in self._nodes]
        for _ in range(max(1, repeat)):
            times = self.module.run_profiled()  # ms per device node, keyed by "+".join(records)
            acc = [0.0] * len(self._nodes)
            carry = 0.0
            for key, ms in times.items():
                if key.startswith("<"):
                    carry += ms  # shadow nodes carry no op: charged to the consumer
                    continue
                # the first of its records that has a graph node (a canonical graph can simplify
                # a plan op away entirely, e.g. a cast back to the clip's own type)
                gi = next((node_of[r] for r in key.split("+") if r in node_of), None)
                if gi is None:
                    carry += ms
                    continue
                acc[gi] += (ms + carry) * 1e-3
                carry = 0.0
            for i, t in enumerate(acc):
                per_node[i].append(t)
        return per_node

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


def create(lib_factory, dev=None, dump_root: Optional[str] = None, granularity: str = "fused") -> GraphModuleDebug:
    """``debug_executor.create`` analogue taking what ``relay.build`` returns."""
    module = lib_factory[lib_factory.mod_name](dev)
    dev_id = int(module.device.index or 0)
    return GraphModuleDebug(module, f"rocm({dev_id})", dump_root, granularity, lib_factory.mod_name)
