"""Cross-host candidate gather over the reference's gRPC contract (SURVEY.md
§8(f) F3: RCCL for co-located shards, gRPC ``CollectScore`` for remote hosts).

Inside a host, the GPUs' shards are merged by RCCL (``Scheduler.comm_init``):
the host's answer for a pod is one ``(node name, TotalScore)``.  Across hosts
every member sends that score, as int32, to the pod's gatherer --
``PodService.CollectScore(SchedulingScore) returns (ScheduleResponse)``
(``dist-scheduler/proto/pod.proto:21-35``) -- and the gatherer's
ScoreEvaluator answers each sender whether its node won
(``grpc_server.go:116-127``, ``scoreevaluator.go:45-126``; here the C++
state machine of ``libksgather.so``, include/ksgather.h).

The messages are built at run time from a FileDescriptorProto equal to
pod.proto's ``ScheduleResponse`` / ``SchedulingScore`` (same package, names,
field numbers and types, so the bytes on the wire are the reference's); the
``NewPod`` stream of the same service is the relay tree's pod ingress, outside
this path.
"""
from __future__ import annotations

import asyncio
import contextlib
import ctypes as C
import threading
from typing import Dict, List, Optional, Sequence, Tuple

import grpc
from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

from . import _abi

SERVICE = "podservice.PodService"
COLLECT_SCORE = f"/{SERVICE}/CollectScore"
GRPC_PORT = 50051  # distpermit.go:87 (the reference hard-codes it)
SCORE_DELAY_S = 5.0  # grpc_server.go:135
TIE_RANDOM, TIE_LOWEST_NAME, TIE_LOWEST_INDEX = 0, 1, 2  # include/ksgather.h


def _messages():
    fd = descriptor_pb2.FileDescriptorProto(name="ksched_pod.proto", package="podservice", syntax="proto3")
    m = fd.message_type.add(name="ScheduleResponse")
    m.field.add(name="permit", number=1, type=descriptor_pb2.FieldDescriptorProto.TYPE_BOOL,
                label=descriptor_pb2.FieldDescriptorProto.LABEL_OPTIONAL, json_name="permit")
    m = fd.message_type.add(name="SchedulingScore")
    for i, (name, typ) in enumerate((("podName", "TYPE_STRING"), ("namespace", "TYPE_STRING"),
                                     ("nodeName", "TYPE_STRING"), ("score", "TYPE_INT32")), start=1):
        m.field.add(name=name, number=i, type=getattr(descriptor_pb2.FieldDescriptorProto, typ),
                    label=descriptor_pb2.FieldDescriptorProto.LABEL_OPTIONAL, json_name=name)
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    get = message_factory.GetMessageClass
    return (get(pool.FindMessageTypeByName("podservice.ScheduleResponse")),
            get(pool.FindMessageTypeByName("podservice.SchedulingScore")))


ScheduleResponse, SchedulingScore = _messages()


def host_score(result, node_names) -> Tuple[str, int]:
    """A host's CollectScore payload for one ks_result: the chosen node's name
    and TotalScore as int32 (distpermit.go:106), or ("", 0) when the host has
    no feasible node (scheduler.go:397-400: score 0 = no candidate)."""
    if result.status != 0 or result.node_index < 0:
        return "", 0
    return node_names[result.node_index], int(result.total_score)


class ScoreEvaluator:
    """ctypes handle on the gatherer state machine (ksg_record_and_wait)."""

    def __init__(self, members: int, delay_s: float = SCORE_DELAY_S, tie: int = TIE_RANDOM, seed: int = 0):
        self.lib = _abi.ksgather_lib()
        self.h = self.lib.ksg_open(members, int(delay_s * 1000), tie, seed)
        if not self.h:
            raise ValueError("ksg_open: bad arguments")
        # Call gate: a thread holds a use of the handle from before it reads it
        # until its C call returns, and close() frees only after every use
        # ended (ksg_shutdown first releases the callers blocked inside), so
        # no call ever reaches a freed evaluator.
        self._gate = threading.Condition()
        self._uses = 0

    @contextlib.contextmanager
    def _use(self, what: str):
        with self._gate:
            if self.h is None:
                raise ValueError(f"{what}: evaluator closed")
            self._uses += 1
            h = self.h
        try:
            yield h
        finally:
            with self._gate:
                self._uses -= 1
                self._gate.notify_all()

    def set_members(self, members: int):
        with self._use("ksg_set_members") as h:
            self.lib.ksg_set_members(h, members)

    def set_node_order(self, names: Sequence[str]):
        """TIE_LOWEST_INDEX: names[i] is global node index i (the hosts' slots end to end)."""
        arr = (C.c_char_p * max(1, len(names)))(*[n.encode() for n in names])
        with self._use("ksg_set_node_order") as h:
            self.lib.ksg_set_node_order(h, arr, len(names))

    def record(self, key: str, node_name: str, score: int):
        """Non-blocking record: (True/False, winner, score) when this score fired
        the evaluation, else ("pending", evaluation id)."""
        buf = C.create_string_buffer(512)
        ws, eid = C.c_int32(), C.c_uint64()
        with self._use("ksg_record") as h:
            r = self.lib.ksg_record(h, key.encode(), node_name.encode(), int(score), C.byref(eid), buf, 512,
                                    C.byref(ws))
        if r < 0:
            raise ValueError("ksg_record: bad arguments or closed")
        if r == 2:
            return "pending", eid.value
        return r == 1, buf.value.decode(), ws.value

    def next_fired(self, timeout_ms: int):
        """(evaluation id, winner, score) of the next evaluation with pending
        records that fired, None on timeout, False once closed."""
        buf = C.create_string_buffer(512)
        eid, ws = C.c_uint64(), C.c_int32()
        try:
            with self._use("ksg_next_fired") as h:
                r = self.lib.ksg_next_fired(h, timeout_ms, C.byref(eid), buf, 512, C.byref(ws))
        except ValueError:
            return False  # closed
        if r < 0:
            return False
        if r == 0:
            return None
        return eid.value, buf.value.decode(), ws.value

    def record_and_wait(self, key: str, node_name: str, score: int) -> Tuple[bool, str, int]:
        """Blocks (without the GIL) until the pod fires; (permit, winner, winner score)."""
        buf = C.create_string_buffer(512)
        ws = C.c_int32()
        with self._use("ksg_record_and_wait") as h:
            r = self.lib.ksg_record_and_wait(h, key.encode(), node_name.encode(), int(score), buf, 512, C.byref(ws))
        if r < 0:
            raise ValueError("ksg_record_and_wait: bad arguments")
        return r == 1, buf.value.decode(), ws.value

    def pending(self) -> int:
        with self._use("ksg_pending") as h:
            return self.lib.ksg_pending(h)

    def close(self):
        """Fires every pending pod (its senders get their answers), refuses
        later calls, and frees the state machine once no call is inside."""
        with self._gate:
            h, self.h = self.h, None
        if not h:
            return
        self.lib.ksg_shutdown(h)  # releases callers blocked in record_and_wait
        with self._gate:
            self._gate.wait_for(lambda: self._uses == 0)
        self.lib.ksg_close(h)


def target_index(key: str, members: Sequence[str], leader: Optional[str] = None) -> int:
    """SchedulerSet.GetTargetForScoring: index into `members` of the gatherer of `key`."""
    lib = _abi.ksgather_lib()
    arr = (C.c_char_p * max(1, len(members)))(*[m.encode() for m in members])
    return lib.ksg_target_index(key.encode(), arr, len(members), leader.encode() if leader else None)


class CollectScoreServer:
    """The gatherer side: PodService.CollectScore on a grpc.aio server.

    A CollectScore RPC records its score without blocking (ksg_record); the
    RPCs of a pod that is still collecting park on asyncio futures, and ONE
    thread (ksg_next_fired) reports every evaluation that fires -- all members
    in, or its delay expired -- to the event loop, which answers each parked
    sender.  In-flight pods are therefore not bounded by a thread pool (the
    reference runs one goroutine per RPC, grpc_server.go:116-127)."""

    def __init__(self, evaluator: ScoreEvaluator, address: str = "127.0.0.1:0", workers: Optional[int] = None):
        del workers  # no per-RPC threads (kept for callers of the former thread-pool server)
        self.evaluator = evaluator
        self._bind = address
        self._waiting: Dict[int, List[Tuple[str, asyncio.Future]]] = {}
        self._loop = asyncio.new_event_loop()
        self._ready = threading.Event()
        self._stopped = threading.Event()
        self._thread = threading.Thread(target=self._serve, name="collect-score", daemon=True)
        self._fired = threading.Thread(target=self._fired_loop, name="collect-score-fired", daemon=True)
        self.port = 0
        self.address = ""
        self._start_error: Optional[BaseException] = None

    # -- event loop thread
    def _serve(self):
        asyncio.set_event_loop(self._loop)
        try:
            self._loop.run_until_complete(self._start())
        except BaseException as e:  # e.g. the address cannot be bound: start() re-raises it
            self._start_error = e
            self._ready.set()
            return
        self._ready.set()
        self._loop.run_forever()

    async def _start(self):
        self.server = grpc.aio.server()
        handler = grpc.unary_unary_rpc_method_handler(
            self._collect, request_deserializer=SchedulingScore.FromString,
            response_serializer=ScheduleResponse.SerializeToString)
        self.server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(SERVICE, {"CollectScore": handler}),))
        self.port = self.server.add_insecure_port(self._bind)
        self.address = f"{self._bind.rsplit(':', 1)[0]}:{self.port}"
        await self.server.start()

    async def _collect(self, req, context):
        r = self.evaluator.record(f"{req.namespace}/{req.podName}", req.nodeName, req.score)
        if r[0] != "pending":
            return ScheduleResponse(permit=r[0])
        fut = self._loop.create_future()  # registered before the loop can run the fire report
        self._waiting.setdefault(r[1], []).append((req.nodeName, fut))
        return ScheduleResponse(permit=await fut)

    def _resolve(self, eval_id: int, winner: str):
        for node, fut in self._waiting.pop(eval_id, []):
            if not fut.done():
                fut.set_result(node == winner)

    # -- the one thread that waits for evaluations to fire
    def _fired_loop(self):
        # every evaluation that has fired is reported before the loop ends,
        # those a closed evaluator fired included (next_fired drains them)
        while True:
            r = self.evaluator.next_fired(200)
            if r is False:  # closed and drained
                break
            if r:
                self._loop.call_soon_threadsafe(self._resolve, r[0], r[1])
            elif self._stopped.is_set():
                break

    def start(self):
        self._thread.start()
        if not self._ready.wait(30):
            raise TimeoutError("CollectScore server did not start within 30 s")
        if self._start_error is not None:
            self._thread.join(5)
            raise self._start_error
        self._fired.start()
        return self

    def stop(self, grace: float = 0.5):
        """Stops serving.  Senders parked on an evaluation that has fired by
        now get their answer -- close the ScoreEvaluator first to fire every
        pending pod with the scores recorded so far; senders still parked after
        `grace` seconds are cancelled (the sender sees an RPC error: no permit,
        as DistPermit treats a failed SendScore)."""
        self._stopped.set()
        self._fired.join(30)  # fired evaluations reported to the loop
        fut = asyncio.run_coroutine_threadsafe(self.server.stop(grace=grace), self._loop)
        try:
            fut.result(30 + grace)
        finally:
            self._loop.call_soon_threadsafe(self._loop.stop)
            self._thread.join(30)


class ScoreClient:
    """The member side (distpermit.SendScore): one cached channel per gatherer."""

    _lock = threading.Lock()
    _channels: dict = {}
    _inflight: set = set()  # fire-and-forget calls (a dropped grpc future cancels its call)

    def __init__(self, address: str):
        with ScoreClient._lock:
            ch = ScoreClient._channels.get(address)
            if ch is None:
                ch = grpc.insecure_channel(address)
                ScoreClient._channels[address] = ch
        self.call = ch.unary_unary(COLLECT_SCORE, request_serializer=SchedulingScore.SerializeToString,
                                   response_deserializer=ScheduleResponse.FromString)

    def send_score(self, pod_name: str, namespace: str, node_name: str, score: int, timeout: float = 30.0) -> bool:
        """The permit for node_name.  Score 0 (no candidate) is sent without
        waiting for the answer, which is a rejection (distpermit.go:111-115)."""
        req = SchedulingScore(podName=pod_name, namespace=namespace, nodeName=node_name, score=int(score))
        if score == 0:
            fut = self.call.future(req, timeout=timeout)
            with ScoreClient._lock:
                ScoreClient._inflight.add(fut)

            def done(f):
                with ScoreClient._lock:
                    ScoreClient._inflight.discard(f)

            fut.add_done_callback(done)
            return False
        try:
            return bool(self.call(req, timeout=timeout).permit)
        except grpc.RpcError:
            return False  # "could not send score. Denying permit"
