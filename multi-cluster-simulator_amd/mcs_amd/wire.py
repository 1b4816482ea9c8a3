"""Wire formats around the placement path: the reference's JSON and protobuf
records, converted to and from the engine's SoA streams and results.

* ``Job`` JSON: ``scheduler.Job`` (pkg/scheduler/scheduler.go:65-73) as the client encodes it
  (``json.NewEncoder(buf).Encode(j)``, pkg/client/server.go:43-46) and the scheduler decodes it
  (``json.NewDecoder(r.Body).Decode(&j)``, pkg/scheduler/server.go:28-30, 57-59, 83-85, 118-120).
  ``streams_from_posts`` turns the POST bodies each cluster received into the engine's
  arrival-ordered streams (the ingestion order of server.go:41,69); ``posts_from_streams`` is the
  client side (client.go:92-102).
* ``Cluster`` JSON: the "/newClient" reply (server.go:139-152).  ``cluster_snapshot`` rebuilds it
  at a simulated second from a run's placements: live counters, ``RunningJobs`` maps and the
  utilization sums.
* Trader protobuf messages (pkg/trader/proto/trader.proto:20-49, resource-channel.proto:27-52) in
  the proto3 binary encoding protobuf-go v1.34.1 (go.mod:20) emits for them: fields in number
  order, implicit-presence zeros omitted, ``optional`` fields present when set, nil elements of a
  repeated message field as empty messages.  ``provide_jobs_batches`` is ProvideJobs' batching of
  Level1 (trader_server.go:69-94, D9) and ``cluster_state`` the Start-stream record
  (trader_server.go:24-47).

Go rules restated (Go 1.21, go.mod:3; encoding/json decode.go and encode.go):

* decode: object keys match field names exactly, else case-insensitively; keys assign in document
  order, so the last key naming a field wins; unknown keys are ignored; ``null`` leaves a field
  unchanged; unsigned fields accept only integer literals in [0, 2^64), ``time.Duration`` integer
  literals in [-2^63, 2^63) ("1.0" and "1e3" are type errors); string fields only JSON strings;
  ``time.Time`` an RFC 3339 string; only the first JSON value of a body is read.  Any error is the
  handler's HTTP 400 (server.go:32-35) and raises ``WireError``.
* encode: fields in declaration order, compact, with ``Encoder``'s HTML escaping (<, >, & as
  \\u003c, \\u003e, \\u0026), U+2028/U+2029 escaped, control characters as \\n, \\r, \\t or \\u00XX,
  and a trailing newline; float32 in the shortest form that round-trips, exponent form below 1e-6
  and from 1e21 up ("1e-7", "1e+21"); NaN and infinities are errors; map keys sorted as strings.

Conversions to the engine apply its input rules: durations are whole seconds (D8), cores and memory
fit uint32 (D7).  Violations raise ``WireError``; nothing is truncated.
"""
from __future__ import annotations

import datetime as _dt
import json
import re
import struct
from dataclasses import dataclass, field, fields
from typing import List, Optional, Sequence, Tuple

import numpy as np

from .cluster import U32_MAX, Cluster

NS_PER_S = 1_000_000_000
U64_MAX = (1 << 64) - 1
I64_MIN, I64_MAX = -(1 << 63), (1 << 63) - 1
ZERO_TIME = "0001-01-01T00:00:00Z"  # time.Time{} as MarshalJSON writes it
BATCH = 20  # ProvideJobs batch size (trader_server.go:75)

# StateType values (scheduler.go:81-86)
READY, RUNNING, WAITING, FINISHED = "Ready", "Running", "Waiting", "Finished"


class WireError(ValueError):
    """A body the reference rejects (HTTP 400), or a value outside the engine's ranges (D7/D8)."""


# ---- encoding/json: decoding ------------------------------------------------------------------
class _Num(str):
    """A JSON number literal kept as text: Go parses it per destination kind."""


class _Obj(list):
    """A JSON object as its (key, value) pairs in document order (duplicates kept)."""


def _reject_constant(name):
    raise WireError(f"invalid character in JSON: {name}")


def _first_value(data):
    """Decoder.Decode: the first JSON value of the body; leading whitespace is skipped and anything
    after the value is not read."""
    if isinstance(data, (bytes, bytearray, memoryview)):
        text = bytes(data).decode("utf-8", errors="replace")  # Go substitutes U+FFFD
    else:
        text = str(data)
    i = len(text) - len(text.lstrip(" \t\r\n"))
    if i == len(text):
        raise WireError("EOF")
    dec = json.JSONDecoder(object_pairs_hook=_Obj, parse_float=_Num, parse_int=_Num,
                           parse_constant=_reject_constant)
    try:
        value, _ = dec.raw_decode(text, i)
    except json.JSONDecodeError as ex:
        raise WireError(f"invalid JSON: {ex.msg} at offset {ex.pos}") from None
    return value


def _kind(v) -> str:
    if isinstance(v, _Num):
        return "number"
    if isinstance(v, str):
        return "string"
    if isinstance(v, bool):
        return "bool"
    if isinstance(v, _Obj):
        return "object"
    if isinstance(v, list):
        return "array"
    return "null"


def _type_error(v, field_name: str, gotype: str) -> WireError:
    return WireError(f"json: cannot unmarshal {_kind(v)} into Go struct field Job.{field_name} of type {gotype}")


def _as_uint(v, name: str) -> int:
    if not isinstance(v, _Num) or not re.fullmatch(r"0|[1-9][0-9]*", v) or int(v) > U64_MAX:
        raise _type_error(v, name, "uint")
    return int(v)


def _as_duration(v, name: str) -> int:
    if not isinstance(v, _Num) or not re.fullmatch(r"-?(0|[1-9][0-9]*)", v) or not I64_MIN <= int(v) <= I64_MAX:
        raise _type_error(v, name, "time.Duration")
    return int(v)


def _as_string(v, name: str) -> str:
    if type(v) is not str:
        raise _type_error(v, name, "string")
    return v


_RFC3339 = re.compile(r"(\d{4})-(\d{2})-(\d{2})T(\d{2}):(\d{2}):(\d{2})(\.\d{1,9})?(Z|[+-]\d{2}:\d{2})")


def _norm_time(text: str) -> str:
    """time.Time UnmarshalJSON then MarshalJSON: RFC 3339 in, RFC 3339 with nanoseconds out
    (fraction trailing zeros trimmed, a zero offset written Z)."""
    m = _RFC3339.fullmatch(text)
    if not m:
        raise WireError(f'parsing time "{text}" as RFC 3339')
    y, mo, d, hh, mi, ss = (int(m.group(k)) for k in range(1, 7))
    frac, off = m.group(7) or "", m.group(8)
    try:  # month, day-of-month and clock ranges (year 0 is valid in Go: check it as leap year 4)
        _dt.datetime(y if y > 0 else 4, mo, d, hh, mi, ss)
    except ValueError as ex:
        raise WireError(f'parsing time "{text}": {ex}') from None
    if off != "Z":
        oh, om = int(off[1:3]), int(off[4:6])
        if oh > 23 or om > 59:
            raise WireError(f'parsing time "{text}": time zone offset out of range')
        if oh == 0 and om == 0:
            off = "Z"
    frac = frac.rstrip("0")
    if frac == ".":
        frac = ""
    return f"{m.group(1)}-{m.group(2)}-{m.group(3)}T{m.group(4)}:{m.group(5)}:{m.group(6)}{frac}{off}"


# ---- encoding/json: encoding ------------------------------------------------------------------
def _jstr(s: str) -> str:
    """encodeState.string with HTML escaping (Go 1.21 encode.go)."""
    out = ['"']
    for ch in s:
        o = ord(ch)
        if ch == '"' or ch == "\\":
            out.append("\\" + ch)
        elif ch in "<>&" or o in (0x2028, 0x2029):
            out.append("\\u%04x" % o)
        elif o < 0x20:
            out.append({"\n": "\\n", "\r": "\\r", "\t": "\\t"}.get(ch, "\\u%04x" % o))
        elif 0xD800 <= o <= 0xDFFF:
            out.append("�")  # not valid UTF-8: Go writes U+FFFD
        else:
            out.append(ch)
    out.append('"')
    return "".join(out)


_F32_LO, _F32_HI = np.float32(1e-6), np.float32(1e21)


def go_float32(x) -> str:
    """encoding/json floatEncoder(32): strconv.AppendFloat(f, 'f' or 'e', -1, 32), the exponent form
    below 1e-6 and from 1e21 up, with "e-07" cleaned to "e-7"."""
    f = np.float32(x)
    if not np.isfinite(f):
        raise WireError(f"json: unsupported value: {float(f)}")
    a = abs(f)
    if a != 0 and (a < _F32_LO or a >= _F32_HI):
        b = np.format_float_scientific(f, unique=True, trim="-", exp_digits=2)
        n = len(b)
        if n >= 4 and b[n - 4] == "e" and b[n - 3] == "-" and b[n - 2] == "0":
            b = b[: n - 2] + b[n - 1]
        return b
    return np.format_float_positional(f, unique=True, trim="-")


# ---- scheduler.Job ----------------------------------------------------------------------------
@dataclass
class Job:
    """scheduler.Job (scheduler.go:65-73); Duration in nanoseconds (time.Duration), WaitTime an
    RFC 3339 string (time.Time)."""

    Id: int = 0
    MemoryNeeded: int = 0
    CoresNeeded: int = 0
    State: str = ""
    Duration: int = 0
    WaitTime: str = ZERO_TIME
    Ownership: str = ""


_JOB_FIELDS = tuple(f.name for f in fields(Job))
_JOB_CONV = {"Id": _as_uint, "MemoryNeeded": _as_uint, "CoresNeeded": _as_uint, "State": _as_string,
             "Duration": _as_duration, "Ownership": _as_string}


def _field_for(key: str) -> Optional[str]:
    if key in _JOB_FIELDS:
        return key
    k = key.casefold()
    for name in _JOB_FIELDS:
        if name.casefold() == k:
            return name
    return None


def decode_job(data) -> Job:
    """json.NewDecoder(body).Decode(&j) (server.go:28-30): WireError where the handler answers 400."""
    v = _first_value(data)
    j = Job()
    if v is None:  # "null": Decode leaves the zero Job and reports no error
        return j
    if not isinstance(v, _Obj):
        raise WireError(f"json: cannot unmarshal {_kind(v)} into Go value of type scheduler.Job")
    err = None
    for key, val in v:
        name = _field_for(key)
        if name is None or val is None:
            continue
        try:
            if name == "WaitTime":
                if type(val) is not str:
                    raise WireError("Time.UnmarshalJSON: input is not a JSON string")
                setattr(j, name, _norm_time(val))
            else:
                setattr(j, name, _JOB_CONV[name](val, name))
        except WireError as ex:  # Go keeps decoding and returns the first type error
            err = err or ex
    if err is not None:
        raise err
    return j


def _job_obj(j: Job) -> str:
    for name in ("Id", "MemoryNeeded", "CoresNeeded"):
        v = getattr(j, name)
        if not 0 <= int(v) <= U64_MAX:
            raise WireError(f"Job.{name} = {v} does not fit Go uint")
    if not I64_MIN <= int(j.Duration) <= I64_MAX:
        raise WireError(f"Job.Duration = {j.Duration} does not fit time.Duration")
    return ('{"Id":%d,"MemoryNeeded":%d,"CoresNeeded":%d,"State":%s,"Duration":%d,"WaitTime":%s,"Ownership":%s}'
            % (int(j.Id), int(j.MemoryNeeded), int(j.CoresNeeded), _jstr(j.State), int(j.Duration),
               _jstr(_norm_time(j.WaitTime)), _jstr(j.Ownership)))


def encode_job(j: Job) -> bytes:
    """json.NewEncoder(buf).Encode(j) (client/server.go:43-46): one compact line."""
    return (_job_obj(j) + "\n").encode("utf-8")


def job_record(j: Job) -> Tuple[int, int, int]:
    """(dur_s, cores, mem) of the engine's job record; D8 whole seconds, D7 uint32 counters."""
    if j.Duration < 0 or j.Duration % NS_PER_S:
        raise WireError(f"job {j.Id}: Duration {j.Duration} ns is not a whole number of seconds >= 0 (D8)")
    d = j.Duration // NS_PER_S
    if d > U32_MAX:
        raise WireError(f"job {j.Id}: Duration {d} s exceeds the engine's uint32 seconds (D8)")
    if j.CoresNeeded > U32_MAX or j.MemoryNeeded > U32_MAX:
        raise WireError(f"job {j.Id}: CoresNeeded/MemoryNeeded exceed the engine's uint32 counters (D7)")
    return d, j.CoresNeeded, j.MemoryNeeded


def streams_from_posts(posts: Sequence[Sequence[Tuple[int, bytes]]]):
    """The bodies each cluster's scheduler received, as (arrival second, body) in arrival order,
    to the engine's CSR streams (job index = position: the ReadyQueue / Level0 order of
    server.go:41,69) and the Go job Ids per cluster (engine job i of cluster k is ids[k][i])."""
    from .engine import JobStreams

    cols = ([], [], [], [])
    ids, off = [], [0]
    for k, cl in enumerate(posts):
        last, kid = 0, []
        for i, (t, body) in enumerate(cl):
            t = int(t)
            if not 0 <= t <= U32_MAX:
                raise WireError(f"cluster {k}: post {i} arrives at {t} s, outside the engine's uint32 clock (D8)")
            if t < last:
                raise WireError(f"cluster {k}: post {i} arrives at {t} s, before {last} s (streams are in arrival order)")
            last = t
            j = decode_job(body)
            d, c, m = job_record(j)
            for col, v in zip(cols, (t, d, c, m)):
                col.append(v)
            kid.append(j.Id)
        off.append(len(cols[0]))
        ids.append(np.array(kid, dtype=np.uint64))
    u32 = [np.array(c, dtype=np.uint32) for c in cols]
    return JobStreams(u32[0], u32[1], u32[2], u32[3], np.array(off, dtype=np.uint64)), ids


def posts_from_streams(streams, ids=None) -> List[List[Tuple[int, bytes]]]:
    """The client side (client.go:92-102, server.go:35-66): job i of cluster k as the body SendJob
    posts at its arrival second; Id = the client's counter (0, 1, ... per cluster) unless given."""
    out = []
    for k in range(len(streams.job_off) - 1):
        s = streams.of(k)
        kid = ids[k] if ids is not None else np.arange(s.stop - s.start)
        rows = []
        for i, (a, d, c, m) in enumerate(zip(streams.arrival[s], streams.dur[s], streams.cores[s], streams.mem[s])):
            j = Job(Id=int(kid[i]), MemoryNeeded=int(m), CoresNeeded=int(c), Duration=int(d) * NS_PER_S)
            rows.append((int(a), encode_job(j)))
        out.append(rows)
    return out


# ---- scheduler.Cluster ("/newClient") -----------------------------------------------------------
def fifo_waited(arrival, start, node) -> np.ndarray:
    """Which jobs of one FIFO cluster went through the WaitQueue (State = WAITING, scheduler.go:266).
    Under SFIFO job i is first tried at max(arrival_i, start_{i-1} + w_{i-1}) (a WaitQueue placement
    sleeps 1 s, :250; a ReadyQueue one does not, :272) and waited iff it started later."""
    n = len(arrival)
    w = np.zeros(n, dtype=bool)
    prev = 0
    for i in range(n):
        if node[i] < 0:  # never placed: the rest of the stream never starts
            w[i:] = node[i:] < 0
            break
        attempt = max(int(arrival[i]), prev)
        w[i] = int(start[i]) > attempt
        prev = int(start[i]) + (1 if w[i] else 0)
    return w


def cluster_snapshot(cluster: Cluster, t: int, arrival, dur, cores, mem, node, start, finish, ids=None,
                     policy: str = "FIFO", epoch_s: int = 0, sampled: bool = True) -> bytes:
    """The "/newClient" body (server.go:139-152) of one cluster at simulated second t, rebuilt from
    a FIFO or DELAY run's placements of its jobs (mcs_read_placements; no trading).

    Every node carries its counters after the releases and decisions of second t (D3), and its
    RunningJobs map (cluster.go:145,154).  The map is keyed by Job.Id, so equal Ids share one entry;
    it is replayed in event order (releases, then decisions in job order; a zero-duration job inserts
    and deletes at once).  Map values are the Job as the scheduler passed it to RunJob: FIFO marks a
    job that went through the WaitQueue "Waiting" (scheduler.go:266); DELAY stamps WaitTime =
    time.Now() at "/delay" (server.go:68), i.e. epoch_s + arrival, in UTC.  With ``sampled`` the
    Cluster's MemoryUtilization / CoreUtilization hold the float32 sums GetResourceUtilization
    leaves there (cluster.go:51-57) at t; otherwise their zero value."""
    n = len(arrival)
    ids = np.arange(n) if ids is None else ids
    nn = len(cluster.Nodes)
    free_c = [nd.CoresAvailable for nd in cluster.Nodes]
    free_m = [nd.MemoryAvailable for nd in cluster.Nodes]
    running = [dict() for _ in range(nn)]
    waited = fifo_waited(arrival, start, node) if policy == "FIFO" else np.zeros(n, dtype=bool)

    def job_of(i):
        wt = ZERO_TIME
        if policy == "DELAY":
            wt = _dt.datetime.fromtimestamp(epoch_s + int(arrival[i]), _dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")
        return Job(Id=int(ids[i]), MemoryNeeded=int(mem[i]), CoresNeeded=int(cores[i]),
                   State=WAITING if waited[i] else "", Duration=int(dur[i]) * NS_PER_S, WaitTime=wt)

    events = []  # (second, phase, order, kind, job): phase 0 releases, 1 decisions
    for i in range(n):
        k = int(node[i])
        if k < 0:
            continue
        if k >= nn:
            raise WireError(f"job {i} placed on node {k}: virtual nodes are not part of a non-trading snapshot")
        s, f = int(start[i]), int(finish[i])
        if s <= t:
            events.append((s, 1, i, "run", i))
            if f > s and f <= t:
                events.append((f, 0, i, "release", i))
    events.sort()
    for _, _, _, kind, i in events:
        k, key = int(node[i]), int(ids[i])
        if kind == "run":
            running[k][key] = i
            free_c[k] = (free_c[k] - int(cores[i])) & U64_MAX
            free_m[k] = (free_m[k] - int(mem[i])) & U64_MAX
            if int(finish[i]) == int(start[i]):  # RunJob sleeps 0: released before the next decision
                running[k].pop(key, None)
                free_c[k] = (free_c[k] + int(cores[i])) & U64_MAX
                free_m[k] = (free_m[k] + int(mem[i])) & U64_MAX
        else:
            running[k].pop(key, None)
            free_c[k] = (free_c[k] + int(cores[i])) & U64_MAX
            free_m[k] = (free_m[k] + int(mem[i])) & U64_MAX

    nodes_js = []
    for k, nd in enumerate(cluster.Nodes):
        rj = ",".join(f"{_jstr(str(key))}:{_job_obj(job_of(i))}"
                      for key, i in sorted(running[k].items(), key=lambda kv: str(kv[0])))
        nodes_js.append('{"Id":%d,"Type":%s,"URL":%s,"Memory":%d,"Cores":%d,"MemoryAvailable":%d,'
                        '"CoresAvailable":%d,"RunningJobs":{%s},"Time":0}'
                        % (nd.Id, _jstr(nd.Type), _jstr(nd.URL), nd.Memory, nd.Cores, free_m[k], free_c[k], rj))
    cu = mu = np.float32(0.0)
    if sampled:
        for k, nd in enumerate(cluster.Nodes):  # node order, float32 (cluster.go:53-57)
            cu = np.float32(cu + np.float32(np.float32(nd.Cores) - np.float32(free_c[k])))
            mu = np.float32(mu + np.float32(np.float32(nd.Memory) - np.float32(free_m[k])))
    tc, tm = cluster.GetTotalResources()
    text = ('{"Id":%d,"Nodes":[%s],"URL":%s,"TotalMemory":%d,"TotalCore":%d,"MemoryUtilization":%s,'
            '"CoreUtilization":%s}\n' % (cluster.Id, ",".join(nodes_js), _jstr(cluster.URL), tm, tc,
                                         go_float32(mu), go_float32(cu)))
    return text.encode("utf-8")


# ---- protobuf (proto3 binary, protobuf-go v1.34.1) ----------------------------------------------
@dataclass
class Duration:
    """google.protobuf.Duration; durationpb.New(d) = {d / 1e9, d % 1e9} (truncated, same sign)."""

    seconds: int = 0
    nanos: int = 0

    @staticmethod
    def from_ns(d: int) -> "Duration":
        q = abs(d) // NS_PER_S
        r = abs(d) % NS_PER_S
        return Duration(-q, -r) if d < 0 else Duration(q, r)

    def to_ns(self) -> int:
        """AsDuration: seconds * 1e9 + nanos, saturated at the int64 range."""
        v = self.seconds * NS_PER_S + self.nanos
        return max(I64_MIN, min(I64_MAX, v))


@dataclass
class ClusterState:  # resource-channel.proto:27-34
    cores_utilization: float = 0.0
    memory_utilization: float = 0.0
    total_cpu: Optional[int] = None
    total_memory: Optional[int] = None
    average_wait_time: float = 0.0


@dataclass
class ContractRequest:  # trader.proto:20-27
    id: int = 0
    cores: int = 0
    memory: int = 0
    time: Optional[Duration] = None
    price: float = 0.0
    trader: str = ""


@dataclass
class ContractResponse:  # trader.proto:29-40
    id: int = 0
    approve: bool = False
    cores: int = 0
    memory: int = 0
    time: Optional[Duration] = None
    price: float = 0.0
    trader: str = ""


@dataclass
class NodeObject:  # trader.proto:42-49
    id: int = 0
    url: str = ""
    cores: int = 0
    memory: int = 0
    time: Optional[Duration] = None


@dataclass
class VirtualNodeRequest:  # resource-channel.proto:36-41
    id: int = 0
    cores: int = 0
    memory: int = 0
    time: Optional[Duration] = None


@dataclass
class PbJob:  # resource-channel.proto:48-52 (trader.Job)
    cores_needed: int = 0
    memory_needed: int = 0
    unix_time_seconds: Optional[Duration] = None


@dataclass
class ProvideJobsResponse:  # resource-channel.proto:45-47; None = a nil element
    jobs: List[Optional[PbJob]] = field(default_factory=list)


SCHEMA = {
    Duration: [(1, "seconds", "int64"), (2, "nanos", "int32")],
    ClusterState: [(1, "cores_utilization", "float"), (2, "memory_utilization", "float"),
                   (3, "total_cpu", "opt_uint32"), (4, "total_memory", "opt_uint32"),
                   (5, "average_wait_time", "double")],
    ContractRequest: [(1, "id", "uint32"), (2, "cores", "uint32"), (3, "memory", "uint32"), (4, "time", Duration),
                      (5, "price", "float"), (6, "trader", "string")],
    ContractResponse: [(1, "id", "uint32"), (2, "approve", "bool"), (3, "cores", "uint32"), (4, "memory", "uint32"),
                       (5, "time", Duration), (6, "price", "float"), (7, "trader", "string")],
    NodeObject: [(1, "id", "uint32"), (2, "url", "string"), (3, "cores", "uint32"), (4, "memory", "uint32"),
                 (5, "time", Duration)],
    VirtualNodeRequest: [(1, "id", "uint32"), (2, "cores", "uint32"), (3, "memory", "uint32"), (4, "time", Duration)],
    PbJob: [(1, "cores_needed", "uint32"), (2, "memory_needed", "uint32"), (3, "unix_time_seconds", Duration)],
    ProvideJobsResponse: [(1, "jobs", [PbJob])],
}
_WIRE_TYPE = {"int64": 0, "int32": 0, "uint32": 0, "opt_uint32": 0, "bool": 0, "float": 5, "double": 1,
              "string": 2}


def _uvarint(v: int) -> bytes:
    v &= U64_MAX
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(num: int, wt: int) -> bytes:
    return _uvarint((num << 3) | wt)


def marshal(msg) -> bytes:
    """proto.Marshal of one of the messages above."""
    out = bytearray()
    for num, name, kind in SCHEMA[type(msg)]:
        v = getattr(msg, name)
        if isinstance(kind, list):  # repeated message; a nil element marshals as an empty message
            for e in v:
                b = marshal(e) if e is not None else b""
                out += _key(num, 2) + _uvarint(len(b)) + b
        elif isinstance(kind, type):  # singular message: present iff set
            if v is not None:
                b = marshal(v)
                out += _key(num, 2) + _uvarint(len(b)) + b
        elif kind == "uint32":
            if not 0 <= int(v) <= U32_MAX:
                raise WireError(f"{type(msg).__name__}.{name} = {v} does not fit uint32")
            if v:
                out += _key(num, 0) + _uvarint(int(v))
        elif kind == "opt_uint32":
            if v is not None:
                if not 0 <= int(v) <= U32_MAX:
                    raise WireError(f"{type(msg).__name__}.{name} = {v} does not fit uint32")
                out += _key(num, 0) + _uvarint(int(v))
        elif kind in ("int32", "int64"):
            lo, hi = (-(1 << 31), (1 << 31) - 1) if kind == "int32" else (I64_MIN, I64_MAX)
            if not lo <= int(v) <= hi:
                raise WireError(f"{type(msg).__name__}.{name} = {v} does not fit {kind}")
            if v:
                out += _key(num, 0) + _uvarint(int(v))  # negative: sign-extended 10-byte varint
        elif kind == "bool":
            if v:
                out += _key(num, 0) + b"\x01"
        elif kind == "float":
            try:
                b = struct.pack("<f", float(v))
            except OverflowError:
                raise WireError(f"{type(msg).__name__}.{name} = {v} does not fit float32") from None
            if b != b"\x00\x00\x00\x00":  # implicit presence: +0.0 is omitted, -0.0 is not
                out += _key(num, 5) + b
        elif kind == "double":
            b = struct.pack("<d", float(v))
            if b != bytes(8):
                out += _key(num, 1) + b
        elif kind == "string":
            if v:
                e = v.encode("utf-8")
                out += _key(num, 2) + _uvarint(len(e)) + e
    return bytes(out)


def _read_uvarint(data: bytes, i: int) -> Tuple[int, int]:
    v, shift = 0, 0
    for n in range(10):
        if i >= len(data):
            raise WireError("unexpected EOF in varint")
        b = data[i]
        i += 1
        v |= (b & 0x7F) << shift
        if b < 0x80:
            if n == 9 and b > 1:
                raise WireError("varint overflows 64 bits")
            return v & U64_MAX, i
        shift += 7
    raise WireError("varint longer than 10 bytes")


def _signed(v: int, bits: int) -> int:
    v &= (1 << bits) - 1
    return v - (1 << bits) if v >> (bits - 1) else v


def _is_set(kind: str, v) -> bool:
    """proto3 implicit presence: a scalar is present iff it differs from the zero value bitwise."""
    if kind == "float":
        return struct.pack("<f", v) != bytes(4)
    if kind == "double":
        return struct.pack("<d", v) != bytes(8)
    return bool(v)


def _merge(a, b):
    """proto.Merge of b into a: scalars present in b overwrite, messages merge, repeated append."""
    for num, name, kind in SCHEMA[type(a)]:
        vb = getattr(b, name)
        if isinstance(kind, list):
            getattr(a, name).extend(vb)
        elif isinstance(kind, type):
            if vb is not None:
                va = getattr(a, name)
                setattr(a, name, vb if va is None else _merge(va, vb))
        elif kind == "opt_uint32":
            if vb is not None:
                setattr(a, name, vb)
        elif _is_set(kind, vb):
            setattr(a, name, vb)
    return a


def unmarshal(cls, data: bytes):
    """proto.Unmarshal into a new message of type ``cls``.  Unknown fields, and known fields with
    a different wire type, are skipped (protobuf-go keeps them as unknown fields)."""
    msg = cls()
    spec = {num: (name, kind) for num, name, kind in SCHEMA[cls]}
    data = bytes(data)
    i = 0
    while i < len(data):
        key, i = _read_uvarint(data, i)
        num, wt = key >> 3, key & 7
        if num == 0:
            raise WireError("invalid field number 0")
        if wt == 0:
            val, i = _read_uvarint(data, i)
        elif wt == 1:
            if i + 8 > len(data):
                raise WireError("unexpected EOF in fixed64")
            val, i = data[i:i + 8], i + 8
        elif wt == 5:
            if i + 4 > len(data):
                raise WireError("unexpected EOF in fixed32")
            val, i = data[i:i + 4], i + 4
        elif wt == 2:
            n, i = _read_uvarint(data, i)
            if i + n > len(data):
                raise WireError("unexpected EOF in length-delimited field")
            val, i = data[i:i + n], i + n
        else:
            raise WireError(f"unsupported wire type {wt}")
        if num not in spec:
            continue
        name, kind = spec[num]
        if isinstance(kind, list):
            if wt == 2:
                getattr(msg, name).append(unmarshal(kind[0], val))
            continue
        if isinstance(kind, type):
            if wt == 2:
                sub = unmarshal(kind, val)
                cur = getattr(msg, name)
                setattr(msg, name, sub if cur is None else _merge(cur, sub))
            continue
        if wt != _WIRE_TYPE[kind]:
            continue
        if kind in ("uint32", "opt_uint32"):
            setattr(msg, name, val & U32_MAX)
        elif kind == "int32":
            setattr(msg, name, _signed(val, 32))
        elif kind == "int64":
            setattr(msg, name, _signed(val, 64))
        elif kind == "bool":
            setattr(msg, name, val != 0)
        elif kind == "float":
            setattr(msg, name, struct.unpack("<f", val)[0])
        elif kind == "double":
            setattr(msg, name, struct.unpack("<d", val)[0])
        elif kind == "string":
            try:
                setattr(msg, name, val.decode("utf-8"))
            except UnicodeDecodeError:
                raise WireError(f"{cls.__name__}.{name}: string field contains invalid UTF-8") from None
    return msg


def provide_jobs_batches(level1: Sequence[Tuple[int, int, int]]) -> List[ProvideJobsResponse]:
    """ProvideJobs (trader_server.go:69-94) over Level1 entries (cores, mem, dur_s): batches of 20;
    the last batch keeps its BATCH - r nil entries (make([]*pb.Job, BATCH), :79), which marshal as
    empty Job messages, so the trader receives them as zero jobs (D9)."""
    out = []
    for i in range(0, len(level1), BATCH):
        batch: List[Optional[PbJob]] = [None] * BATCH
        for jj, (c, m, d) in enumerate(level1[i:i + BATCH]):
            batch[jj] = PbJob(cores_needed=int(c) & U32_MAX, memory_needed=int(m) & U32_MAX,
                              unix_time_seconds=Duration.from_ns(int(d) * NS_PER_S))
        out.append(ProvideJobsResponse(batch))
    return out


def cluster_state(cu: float, mu: float, avg_wait_ms: float, totals: Optional[Tuple[int, int]] = None) -> ClusterState:
    """One Start-stream record (trader_server.go:24-47): totals only on the first message after a
    cluster change (:28-34), utilization and WaitTime.GetAverage() on every message."""
    tc, tm = totals if totals is not None else (None, None)
    return ClusterState(cores_utilization=float(np.float32(cu)), memory_utilization=float(np.float32(mu)),
                        total_cpu=tc, total_memory=tm, average_wait_time=float(avg_wait_ms))


__all__ = ["Job", "WireError", "decode_job", "encode_job", "job_record", "streams_from_posts",
           "posts_from_streams", "fifo_waited", "cluster_snapshot", "go_float32", "Duration", "ClusterState",
           "ContractRequest", "ContractResponse", "NodeObject", "VirtualNodeRequest", "PbJob",
           "ProvideJobsResponse", "marshal", "unmarshal", "provide_jobs_batches", "cluster_state",
           "ZERO_TIME", "NS_PER_S", "READY", "RUNNING", "WAITING", "FINISHED"]
