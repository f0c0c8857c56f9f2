"""``graph_executor.GraphModule`` surface (python/tvm/contrib/graph_executor.py:114-351)
plus the trace capture the reference only sketches (README.md:6,16) and the debug
executor's per-node dump (python/tvm/contrib/debugger/debug_executor.py:210-347).

    lib = relay.build(mod, target="mi355x", params=params)
    m = graph_executor.GraphModule(lib["default"](tachikoma_amd.rocm(0)))
    m.set_input("data", x); m.run(); y = m.get_output(0).numpy()
    m.dump_trace("model.tkt")             # every op output of the last run
    m.run(trace=True)                     # run with overlapped D2H capture
"""
from __future__ import annotations

import json
import time
from typing import Any, Dict, List, Optional

import numpy as np

from .. import _lib
from .. import trace_format as tf
from ..relay.device_module import DeviceModule


class NDArrayView:
    """What get_output returns: ``.numpy()`` like tvm.nd.NDArray."""

    def __init__(self, t):
        self._t = t

    def numpy(self) -> np.ndarray:
        return self._t.detach().cpu().numpy()

    @property
    def shape(self):
        return tuple(self._t.shape)

    @property
    def dtype(self):
        return str(self._t.dtype).replace("torch.", "")

    def torch(self):
        return self._t


def _as_bytes(t):
    import torch
    return t.reshape(-1).view(torch.uint8)


class TraceCapture:
    """Pinned host image of one trace shard; device→host copies land at final offsets."""

    def __init__(self, module: DeviceModule, meta: Dict[str, Any]):
        import torch
        self.module = module
        plan = module.plan
        params = [(t.name, t.shape, t.dtype) for t in plan.params]
        records = [(t.name, t.shape, t.dtype) for t in plan.records]
        self.meta = dict(meta)
        self.layout = tf.TraceLayout.compute(tf.header_json(self.meta), params, records)
        self.image = torch.empty(self.layout.total, dtype=torch.uint8, pin_memory=True)
        self.ptr = self.image.data_ptr()
        self.layout.write_headers(self.ptr, self.layout.total)
        # params once, from the device copies (again after load_params: refresh_params)
        self.param_offsets = {p[0]: (off, p[1], p[2]) for p, off in zip(params, self.layout.param_offsets)}
        self.refresh_params(list(self.param_offsets))
        self.record_offsets = dict(zip([r[0] for r in records], self.layout.record_offsets))
        self.host_dst = module.host_dst_array({n: self.ptr + off for n, off in self.record_offsets.items()})
        self.capture_stream = torch.cuda.Stream(device=module.device)

    def refresh_params(self, names) -> None:
        """Copy the named params' device buffers into the params section (synchronous)."""
        for name in names:
            off, shape, dtype = self.param_offsets[name]
            self._host_bytes(off, shape, dtype).copy_(_as_bytes(self.module.buffers[name]))

    def _host_bytes(self, off: int, shape, dtype: str):
        """Byte view of a payload (NDArray-list payloads are not element-aligned)."""
        nbytes = int(np.prod(shape, dtype=np.int64)) * np.dtype(dtype).itemsize
        return self.image[off:off + nbytes]

    def update_meta(self, **kw) -> None:
        self.meta.update(kw)
        text = tf.header_json(self.meta)
        old = self.layout.json_text
        if len(text.rstrip()) > len(old):
            raise _lib.TachikomaError("trace header grew beyond its reserved slack")
        text = text.rstrip().ljust(len(old))
        self.layout.json_text = text
        self.image[56:56 + len(text)].copy_(__import__("torch").frombuffer(bytearray(text.encode()),
                                                                           dtype=__import__("torch").uint8))

    def capture_inputs(self, stream) -> None:
        """Copy the graph inputs (recorded first) on the capture stream."""
        import torch
        self.capture_stream.wait_stream(stream)
        with torch.cuda.stream(self.capture_stream):
            for t in self.module.plan.inputs:
                self._host_bytes(self.record_offsets[t.name], t.shape, t.dtype).copy_(
                    _as_bytes(self.module.buffers[t.name]), non_blocking=True)

    def synchronize(self) -> None:
        self.capture_stream.synchronize()

    def write(self, path: str) -> None:
        tf.write_file(path, self.ptr, self.layout.total)

    def bytes(self) -> memoryview:
        return memoryview(self.image.numpy())


class BenchmarkResult:
    """Runtimes from benchmarking, in seconds (python/tvm/runtime/module.py:34-98): ``results``
    and their mean / std / median / min / max."""

    def __init__(self, results):
        self.results = list(results)
        self.mean = float(np.mean(self.results))
        self.std = float(np.std(self.results))
        self.median = float(np.median(self.results))
        self.min = float(np.min(self.results))
        self.max = float(np.max(self.results))

    def __repr__(self):
        return (f"BenchmarkResult(min={self.min}, mean={self.mean}, median={self.median}, max={self.max}, "
                f"std={self.std}, results={self.results})")

    def __str__(self):
        head = "".join(f"{h:^12} " for h in ("mean (ms)", "median (ms)", "max (ms)", "min (ms)", "std (ms)"))
        vals = "".join(f"{v * 1000:^12.4f} " for v in (self.mean, self.median, self.max, self.min, self.std))
        return f"Execution time summary:\n{head}\n{vals}\n"


def time_evaluator(fn, device, number: int, repeat: int, min_repeat_ms: int = 0,
                   limit_zero_time_iterations: int = 100, cooldown_interval_ms: int = 0,
                   repeats_to_cooldown: int = 1, device_timer: bool = True):
    """``WrapTimeEvaluator`` (src/runtime/profiling.cc): one warm-up call, then ``repeat``
    measurements of ``number`` back-to-back calls each (seconds per call).  A measurement shorter
    than ``min_repeat_ms`` is redone with ``number`` grown (x1.618 at least, to the count the last
    one implies, as the reference does); a zero-time one at most ``limit_zero_time_iterations``
    times.  Device timer: HIP events on the device's current stream around the calls (the
    reference's Timer on ROCm); else wall clock with a device synchronize on both sides."""
    import torch
    stream = torch.cuda.current_stream(device)
    fn()
    torch.cuda.synchronize(device)
    out = []
    for r in range(max(1, repeat)):
        n = max(1, int(number))
        zeros = 0
        while True:
            if device_timer:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(n):
                    fn()
                e1.record(stream)
                e1.synchronize()
                ms = e0.elapsed_time(e1)
            else:
                torch.cuda.synchronize(device)
                t0 = time.perf_counter()
                for _ in range(n):
                    fn()
                torch.cuda.synchronize(device)
                ms = (time.perf_counter() - t0) * 1e3
            if ms <= 0.0 and zeros < limit_zero_time_iterations:
                zeros += 1
                continue
            if ms >= (min_repeat_ms or 0) or ms <= 0.0:
                break
            n = max(int(min_repeat_ms / (ms / n) + 1), int(n * 1.618))
        out.append(ms * 1e-3 / n)
        if cooldown_interval_ms and repeats_to_cooldown and (r + 1) % repeats_to_cooldown == 0:
            time.sleep(cooldown_interval_ms * 1e-3)
    return out


class GraphModule:
    def __init__(self, module: DeviceModule):
        self.module = module
        self.plan = module.plan
        self._capture: Optional[TraceCapture] = None
        self._meta = {"format": "tachikoma-trace", "version": tf.TRACE_VERSION, "model": "graph",
                      "target": "mi355x", "sample_offset": 0, "rank": 0, "world": 1,
                      "semantics": {"reference": "tvm llvm target without -mcpu", "requantize_compute_dtype":
                                    _compute_dtypes(self.plan), "rounding_default": "UPWARD"},
                      "inputs": [t.name for t in self.plan.inputs],
                      "params": [t.name for t in self.plan.params],
                      "outputs": list(self.plan.outputs),
                      "ops": [o.describe() for o in self.plan.ops]}
        if self.plan.inputs:
            self._meta["n_samples"] = int(self.plan.inputs[0].shape[0]) if self.plan.inputs[0].shape else 1

    def close(self) -> None:
        """Wait for the device, then release the native module and the pinned trace image.  Call it
        (or use the module as a context manager) before the process exits; an atexit hook closes
        any module left open (device_module.close_all)."""
        self.module.close()
        if self._capture is not None:
            self._capture.capture_stream.synchronize()
            self._capture = None

    def __enter__(self) -> "GraphModule":
        return self

    def __exit__(self, *exc) -> None:
        self.close()

    # -- reference surface -------------------------------------------------
    def set_input(self, key=None, value=None, **params):
        """graph_executor.py:166-197: ``key`` (name or input index) = ``value`` plus keyword
        params; every shape is checked before the first write, and the writes wait for the
        last traced run's copies (tk_module_wait_capture)."""
        vals = {}
        if key is not None:
            vals[self.plan.inputs[key].name if isinstance(key, int) else key] = value
        vals.update(params)
        self.module.set_inputs(vals)

    def run(self, trace: bool = False, **inputs):
        import torch
        if inputs:
            self.set_input(**inputs)
        stream = torch.cuda.current_stream(self.module.device)
        if trace:
            cap = self.trace_capture()
            cap.capture_inputs(stream)
            self.module.run(stream, cap.capture_stream, cap.host_dst)
        else:
            self.module.run(stream)

    def pick_run_mode(self, steps: int = 2) -> Dict[str, Any]:
        """Submission find step for traced runs on this host: times ``steps`` traced runs issued
        node by node from the host (tk_module_run) and as one replayed HIP graph
        (tk_module_run_graph), and keeps the faster.  On a healthy host the host-issued copies
        reach the SDMA rate and win by ~5 % (profiles/r03n_run_modes.txt); on a host that issues
        the ~300 calls of a step slowly, the graph's single launch does — but such hosts can be
        slow only intermittently (profiles/r03r_run_modes_slow_host.txt: 454 vs 186 op-traces/s
        on one box), which two timed steps may not catch, so bench.py and trace jobs default to the
        graph.  Results are identical either way."""
        import time
        import torch
        times = {}
        for use_graph in (False, True):
            self.module.use_graph = use_graph
            self.run(trace=True)  # warm-up (a graph run captures and instantiates here)
            self.trace_capture().synchronize()
            torch.cuda.synchronize(self.module.device)
            t0 = time.perf_counter()
            for _ in range(max(1, steps)):
                self.run(trace=True)
            self.trace_capture().synchronize()
            torch.cuda.synchronize(self.module.device)
            times[use_graph] = (time.perf_counter() - t0) / max(1, steps)
        self.module.use_graph = times[True] < times[False]
        return {"host_issued_ms": round(times[False] * 1e3, 2), "graph_ms": round(times[True] * 1e3, 2),
                "chosen": "graph" if self.module.use_graph else "host-issued"}

    def get_num_outputs(self) -> int:
        return len(self.plan.outputs)

    def get_input_index(self, name: str) -> int:
        """graph_executor.py:247-260: the input's index, -1 when no input has that name."""
        return next((i for i, t in enumerate(self.plan.inputs) if t.name == name), -1)

    def get_input_info(self):
        """graph_executor.py:262-287: ({input: shape}, {input: dtype}) of the graph inputs (the
        arg nodes that are not params)."""
        return ({t.name: tuple(int(d) for d in t.shape) for t in self.plan.inputs},
                {t.name: t.dtype for t in self.plan.inputs})

    def debug_get_output(self, node, out=None):
        """graph_executor.py:305-316: only the debug executor runs a graph up to a node."""
        raise NotImplementedError("Please use debugger.debug_executor as graph_executor instead.")

    def share_params(self, other: "GraphModule", params_bytes: bytes) -> None:
        """graph_executor.py:328-339 (GraphExecutor::ShareParams, graph_executor.cc:293-310): take
        the params named in ``params_bytes`` (only the names are read) from ``other``, a module of
        the same graph.  The reference aliases the other executor's storage; here each node's
        tensors are the module's own device buffers, bound into its native node list, so the values
        are copied device to device (no host round trip) and the buffers derived from them (packed
        MFMA weights, weight sums) re-derived.  Every name must be a param of both modules with the
        same shape and dtype, checked before the first copy."""
        names = list(tf.parse_ndarray_list(params_bytes, copy=False))
        mine = {t.name: t for t in self.plan.params}
        theirs = {t.name: t for t in other.plan.params}
        sel = {}
        for name in names:
            if name not in mine or name not in theirs:
                raise _lib.TachikomaError(f"share_params: {name} is not a param of both modules")
            a, b = mine[name], theirs[name]
            if tuple(a.shape) != tuple(b.shape) or a.dtype != b.dtype:
                raise _lib.TachikomaError(f"share_params: {name} is {b.dtype}{list(b.shape)} in the other module, "
                                          f"{a.dtype}{list(a.shape)} here")
            sel[name] = other.module.buffers[name]
        self.module.set_inputs(sel)
        if self._capture is not None:
            self._capture.refresh_params([n for n in sel if n in self._capture.param_offsets])

    _FUNCTIONS = ("set_input", "run", "get_output", "get_input", "get_num_outputs", "get_num_inputs",
                  "load_params", "share_params", "get_input_index", "get_input_info", "debug_get_output")

    def __getitem__(self, key: str):
        """graph_executor.py:341-349: the module function ``key`` (module["run"]() etc.)."""
        if key not in self._FUNCTIONS:
            raise AttributeError(f"Module has no function '{key}'")
        return getattr(self, key)

    def benchmark(self, device=None, func_name: str = "run", repeat: int = 5, number: int = 5,
                  min_repeat_ms=None, limit_zero_time_iterations: int = 100, end_to_end: bool = False,
                  cooldown_interval_ms: int = 0, repeats_to_cooldown: int = 1, **kwargs) -> BenchmarkResult:
        """graph_executor.py:351-459: runtimes of ``func_name`` (seconds per call), ``repeat``
        results of ``number`` calls each, timed with device timers (HIP events) so that input
        transfers are not counted.  ``kwargs`` are set as inputs first (not timed).  With
        ``end_to_end`` every call also copies ``kwargs`` host -> device and the outputs back,
        timed by the wall clock."""
        from ..relay.device_module import _as_torch_device
        dev = self.module.device if device is None else _as_torch_device(device)
        min_ms = 0 if min_repeat_ms is None else min_repeat_ms
        if end_to_end:
            host = {k: np.asarray(v.numpy() if hasattr(v, "numpy") else v) for k, v in kwargs.items()}

            def call():
                if host:
                    self.set_input(**host)
                self.run()
                for i in range(self.get_num_outputs()):
                    self.get_output(i).numpy()
            return BenchmarkResult(time_evaluator(call, dev, number, repeat, min_ms, limit_zero_time_iterations,
                                                  cooldown_interval_ms, repeats_to_cooldown, device_timer=False))
        if kwargs:
            self.set_input(**kwargs)
        fn = self[func_name]
        return BenchmarkResult(time_evaluator(fn, dev, number, repeat, min_ms, limit_zero_time_iterations,
                                              cooldown_interval_ms, repeats_to_cooldown))

    def get_num_inputs(self) -> int:
        return len(self.plan.inputs)

    def get_input(self, key) -> NDArrayView:
        if isinstance(key, int):
            key = self.plan.inputs[key].name
        return NDArrayView(self.module.buffers[key])

    def get_output(self, index: int, out=None) -> NDArrayView:
        t = self.module.buffers[self.plan.outputs[index]]
        if out is not None:
            out[...] = t.cpu().numpy()
            return out
        return NDArrayView(t)

    def load_params(self, params_bytes: bytes) -> None:
        """``GraphModule.load_params`` (python/tvm/contrib/graph_executor.py:318-327 →
        GraphExecutor::LoadParams, graph_executor.cc:283-291): an NDArray-list blob
        (file_utils.cc:184-206).  Names that are not graph inputs or params are skipped, like
        the reference; every other entry must match its buffer's shape and dtype, and all of
        them are checked before the first buffer is written.  The build-time buffers derived
        from a param (packed MFMA weights and weight sums) are re-derived on the device, and the
        params section of the trace image is refreshed."""
        known = {t.name: t for t in list(self.plan.inputs) + list(self.plan.params)}
        sel = {}
        for name, arr in tf.parse_ndarray_list(params_bytes, copy=True).items():
            t = known.get(name)
            if t is None:
                continue
            if tuple(arr.shape) != tuple(t.shape) or str(arr.dtype) != t.dtype:
                raise _lib.TachikomaError(f"load_params: {name} is {arr.dtype}{list(arr.shape)}, "
                                          f"the graph expects {t.dtype}{list(t.shape)}")
            sel[name] = arr
        self.module.set_inputs(sel)
        if self._capture is not None:
            self._capture.refresh_params([n for n in sel if n in self._capture.param_offsets])

    # -- trace / debug surface ---------------------------------------------
    def get_node_output(self, name: str) -> NDArrayView:
        return NDArrayView(self.module.buffers[name])

    def node_names(self) -> List[str]:
        return [o.name for o in self.plan.ops]

    def trace_capture(self) -> TraceCapture:
        if self._capture is None:
            self._capture = TraceCapture(self.module, self._meta)
        return self._capture

    def set_trace_meta(self, **kw) -> None:
        self._meta.update(kw)
        if self._capture is not None:
            self._capture.update_meta(**kw)

    def dump_trace(self, path: str, sample_offset: Optional[int] = None) -> str:
        """Write the trace of the last run (re-runs with capture if the last run was not traced)."""
        import torch
        if sample_offset is not None:
            self.set_trace_meta(sample_offset=int(sample_offset))
        stream = torch.cuda.current_stream(self.module.device)
        cap = self.trace_capture()
        cap.capture_inputs(stream)
        self.module.run(stream, cap.capture_stream, cap.host_dst)
        cap.synchronize()
        cap.write(path)
        return path

    def trace_digest(self) -> int:
        """u64 digest of the last run's records, computed on the device
        (equals trace_format.trace_file_digest of the dumped trace)."""
        import torch
        d = self.module.records_digest(torch.cuda.current_stream(self.module.device))
        return int(d.item()) & 0xFFFFFFFFFFFFFFFF

    def profile(self) -> Dict[str, float]:
        """Per-node device time in ms (GraphExecutorDebug::RunIndividual analogue)."""
        return self.module.run_profiled()

    def chrome_trace(self, path: str) -> None:
        """Chrome trace JSON in the debug executor's schema (debug_result.py:151-189)."""
        timings = self.profile()
        events, t = [], 0.0
        for name, ms in timings.items():
            us = ms * 1e3  # Chrome trace "ts" is in microseconds (debug_result.py:151-189)
            events.append({"name": name, "cat": "Op", "ph": "B", "ts": t, "pid": 1, "tid": 1})
            events.append({"name": name, "cat": "Op", "ph": "E", "ts": t + us, "pid": 1, "tid": 1})
            t += us
        with open(path, "w") as f:
            json.dump({"traceEvents": events, "displayTimeUnit": "ns"}, f)


def _compute_dtypes(plan) -> str:
    """The requantize compute dtype(s) the plan's ops were built with (the trace header's claim):
    "int64" (the pinned default), "float32" / "float64", or a "+"-joined list when mixed."""
    cds = sorted({o.attrs.get("compute_dtype", "int64") for o in plan.ops if "compute_dtype" in o.attrs})
    return "+".join(cds) if cds else "int64"


def create(lib_factory, dev=None) -> GraphModule:
    return GraphModule(lib_factory["default"](dev))
