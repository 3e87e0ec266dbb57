"""Pure-Python Kafka client on ``protocol.py`` (no Kafka library is available offline).

* ``KafkaConnection`` -- one TCP connection, request/response by correlation id
  (requests are serialised per connection; each client object owns its connections).
* ``KafkaClient``     -- bootstrap + metadata cache + connections per broker.
* ``Producer``        -- murmur2 partitioner for keyed records, round-robin otherwise,
  linger-free per-call batching (``send_many``), acks=all.
* ``GroupConsumer``   -- consumer-group member (FindCoordinator, JoinGroup with the
  ``range`` assignor computed by the leader, SyncGroup, background Heartbeat,
  LeaveGroup), Fetch from committed offsets (``auto.offset.reset`` earliest/latest),
  **out-of-order commit tracking**: per partition the committed offset advances only
  through the contiguous prefix of acknowledged offsets (``KafkaConsumerWrapper.java:203-277``).
* ``PartitionReader`` -- assign-all, no group; starts at earliest / latest / absolute
  per-partition offsets (gateway readers, ``KafkaReaderWrapper.java:60-150``).
* admin helpers: create / delete topics.
"""
from __future__ import annotations

import itertools
import logging
import random
import socket
import struct
import threading
import time
import uuid
from typing import Any, Callable, Dict, List, Optional, Tuple

from . import protocol as P

log = logging.getLogger(__name__)


class KafkaError(Exception):
    def __init__(self, code: int, msg: str = ""):
        super().__init__(f"Kafka error {code} {msg}")
        self.code = code


class KafkaConnection:
    def __init__(self, host: str, port: int, client_id: str, timeout: float = 30.0, security=None):
        sock = socket.create_connection((host, port), timeout=timeout)
        sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        if security is not None and security.tls:
            sock = security.ssl_context().wrap_socket(sock, server_hostname=host)
        self.sock = sock
        self.client_id = client_id
        self._corr = itertools.count(1)
        self._lock = threading.Lock()
        if security is not None and security.sasl:
            self._sasl(security)

    def _sasl(self, security) -> None:
        """SaslHandshake v1 + SaslAuthenticate v0 (KIP-152): PLAIN (one message) or
        SCRAM-SHA-256/512 (client-first / client-final, server signature verified)."""
        from .security import SCRAM_MECHANISMS, ScramClient, ScramError
        r = self.request(P.SASL_HANDSHAKE, {"mechanism": security.mechanism})
        if r["error"] != P.NONE:
            self.close()
            raise KafkaError(r["error"], f"SASL mechanism {security.mechanism} not enabled; broker offers "
                                         f"{r['mechanisms']}")

        def auth(msg: bytes) -> bytes:
            r = self.request(P.SASL_AUTHENTICATE, {"auth_bytes": msg})
            if r["error"] != P.NONE:
                self.close()
                raise KafkaError(r["error"], f"SASL authentication failed: {r.get('error_message')}")
            return bytes(r.get("auth_bytes") or b"")

        if security.mechanism in SCRAM_MECHANISMS:
            sc = ScramClient(security.mechanism, security.username or "", security.password or "")
            try:
                sc.verify(auth(sc.final(auth(sc.first()))))
            except ScramError as e:
                self.close()
                raise KafkaError(P.SASL_AUTHENTICATION_FAILED, f"SCRAM: {e}") from e
            return
        auth(security.plain_token())

    def _recv_exact(self, n: int) -> bytes:
        buf = bytearray()
        while len(buf) < n:
            chunk = self.sock.recv(n - len(buf))
            if not chunk:
                raise ConnectionError("kafka connection closed")
            buf += chunk
        return bytes(buf)

    def request(self, api_key: int, body: Dict[str, Any], timeout: Optional[float] = None) -> Dict[str, Any]:
        with self._lock:
            corr = next(self._corr)
            self.sock.settimeout(timeout or 30.0)
            self.sock.sendall(P.request_frame(api_key, corr, self.client_id, body))
            n = struct.unpack(">i", self._recv_exact(4))[0]
            payload = self._recv_exact(n)
        rc = struct.unpack_from(">i", payload, 0)[0]
        if rc != corr:
            raise ConnectionError(f"correlation id mismatch {rc} != {corr}")
        return P.Reader(payload, 4).read(P.RESP[api_key])

    def close(self) -> None:
        try:
            self.sock.close()
        except OSError:
            pass


class KafkaClient:
    def __init__(self, bootstrap_servers: str, client_id: str = "langstream-amd", security=None):
        self.bootstrap = [(h.rsplit(":", 1)[0], int(h.rsplit(":", 1)[1]))
                          for h in str(bootstrap_servers).split(",") if h.strip()]
        self.client_id = client_id
        self.security = security
        self._conns: Dict[Tuple[str, int], KafkaConnection] = {}
        self.brokers: Dict[int, Tuple[str, int]] = {}
        self.partitions: Dict[str, Dict[int, int]] = {}  # topic -> partition -> leader
        self._lock = threading.RLock()

    def conn(self, addr: Tuple[str, int]) -> KafkaConnection:
        with self._lock:
            c = self._conns.get(addr)
            if c is None:
                c = KafkaConnection(addr[0], addr[1], self.client_id, security=self.security)
                self._conns[addr] = c
            return c

    def any_conn(self) -> KafkaConnection:
        last = None
        for addr in list(self.brokers.values()) + self.bootstrap:
            try:
                return self.conn(addr)
            except OSError as e:
                last = e
        raise ConnectionError(f"no kafka broker reachable: {last}")

    def refresh_metadata(self, topics: Optional[List[str]] = None) -> None:
        r = self.any_conn().request(P.METADATA, {"topics": topics})
        with self._lock:
            self.brokers = {b["node_id"]: (b["host"], b["port"]) for b in r["brokers"]}
            for t in r["topics"]:
                if t["error"] == P.NONE:
                    self.partitions[t["name"]] = {p["partition"]: p["leader"] for p in t["partitions"]}

    def leader_conn(self, topic: str, partition: int) -> KafkaConnection:
        if topic not in self.partitions:
            self.refresh_metadata([topic])
        leader = self.partitions.get(topic, {}).get(partition)
        if leader is None:
            raise KafkaError(P.UNKNOWN_TOPIC_OR_PARTITION, f"{topic}/{partition}")
        return self.conn(self.brokers[leader])

    def num_partitions(self, topic: str) -> int:
        if topic not in self.partitions:
            self.refresh_metadata([topic])
        n = len(self.partitions.get(topic, {}))
        if n == 0:
            raise KafkaError(P.UNKNOWN_TOPIC_OR_PARTITION, topic)
        return n

    # ---------------------------------------------------------------- admin
    def create_topic(self, name: str, partitions: int = 1, replication: int = 1,
                     configs: Optional[Dict[str, str]] = None) -> bool:
        r = self.any_conn().request(P.CREATE_TOPICS, {"topics": [
            {"name": name, "num_partitions": partitions, "replication_factor": replication, "assignments": [],
             "configs": [{"name": k, "value": str(v)} for k, v in (configs or {}).items()]}], "timeout": 30000})
        err = r["topics"][0]["error"]
        if err not in (P.NONE, P.TOPIC_ALREADY_EXISTS):
            raise KafkaError(err, f"create topic {name}")
        self.refresh_metadata([name])
        return err == P.NONE

    def describe_topic_configs(self, name: str) -> Dict[str, Optional[str]]:
        """DescribeConfigs (v0) of a topic: {config name: value} (Admin.describeConfigs)."""
        r = self.any_conn().request(P.DESCRIBE_CONFIGS, {"resources": [
            {"type": P.RESOURCE_TOPIC, "name": name, "config_names": None}]})
        res = r["resources"][0]
        if res["error"] != P.NONE:
            raise KafkaError(res["error"], f"describe configs {name}: {res.get('error_message')}")
        return {c["name"]: c["value"] for c in res["configs"]}

    def list_topics(self) -> List[str]:
        """Admin.listTopics: every topic the cluster's metadata names."""
        r = self.any_conn().request(P.METADATA, {"topics": None})
        return sorted(t["name"] for t in r["topics"] if t["error"] == P.NONE)

    def delete_topic(self, name: str) -> None:
        self.any_conn().request(P.DELETE_TOPICS, {"topics": [name], "timeout": 30000})
        with self._lock:
            self.partitions.pop(name, None)

    def list_offsets(self, topic: str, timestamp: int) -> Dict[int, int]:
        """timestamp -1 = latest, -2 = earliest."""
        out = {}
        for p in range(self.num_partitions(topic)):
            r = self.leader_conn(topic, p).request(P.LIST_OFFSETS, {"replica_id": -1, "topics": [
                {"name": topic, "partitions": [{"partition": p, "timestamp": timestamp}]}]})
            out[p] = r["topics"][0]["partitions"][0]["offset"]
        return out

    def fetch(self, topic: str, offsets: Dict[int, int], max_wait_ms: int = 500, max_bytes: int = 4 << 20):
        """-> {partition: (high_watermark, [(offset, ts, key, value, headers)])}"""
        by_leader: Dict[int, List[int]] = {}
        if topic not in self.partitions:
            self.refresh_metadata([topic])
        for p in offsets:
            by_leader.setdefault(self.partitions[topic][p], []).append(p)
        out = {}
        for leader, parts in by_leader.items():
            r = self.conn(self.brokers[leader]).request(P.FETCH, {
                "replica_id": -1, "max_wait": max_wait_ms, "min_bytes": 1, "max_bytes": max_bytes, "isolation": 0,
                "topics": [{"name": topic, "partitions": [{"partition": p, "offset": offsets[p],
                                                           "max_bytes": max_bytes} for p in parts]}]},
                timeout=max_wait_ms / 1000.0 + 30)
            for t in r["topics"]:
                for pr in t["partitions"]:
                    if pr["error"] not in (P.NONE,):
                        raise KafkaError(pr["error"], f"fetch {topic}/{pr['partition']}")
                    recs = [x for x in P.decode_batches(pr["records"]) if x[0] >= offsets[pr["partition"]]]
                    out[pr["partition"]] = (pr["hw"], recs)
        return out

    def close(self) -> None:
        with self._lock:
            for c in self._conns.values():
                c.close()
            self._conns.clear()


class Producer:
    def __init__(self, client: KafkaClient, topic: str, codec: int = 0):
        self.client = client
        self.topic = topic
        self.codec = codec
        self._rr = itertools.count(random.randrange(1 << 16))

    def partition(self, key: Optional[bytes]) -> int:
        n = self.client.num_partitions(self.topic)
        if key is None:
            return next(self._rr) % n
        return P.partition_for_key(key, n)

    def send_many(self, records: List[Tuple[Optional[bytes], Optional[bytes], List[Tuple[str, bytes]], int]]):
        by_part: Dict[int, list] = {}
        for r in records:
            by_part.setdefault(self.partition(r[0]), []).append(r)
        offsets = []
        for p, recs in by_part.items():
            r = self.client.leader_conn(self.topic, p).request(P.PRODUCE, {
                "transactional_id": None, "acks": -1, "timeout": 30000,
                "topics": [{"name": self.topic, "partitions": [{"partition": p,
                                                                "records": P.encode_batch(0, recs, self.codec)}]}]})
            pr = r["topics"][0]["partitions"][0]
            if pr["error"] != P.NONE:
                raise KafkaError(pr["error"], f"produce {self.topic}/{p}")
            offsets.append((p, pr["base_offset"]))
        return offsets

    def send(self, key, value, headers, ts) -> Tuple[int, int]:
        return self.send_many([(key, value, headers, ts)])[0]


def range_assign(members: Dict[str, List[str]], partitions: Dict[str, int]) -> Dict[str, Dict[str, List[int]]]:
    """Kafka RangeAssignor: per topic, sorted members get contiguous partition ranges."""
    out: Dict[str, Dict[str, List[int]]] = {m: {} for m in members}
    for topic, n in partitions.items():
        subs = sorted(m for m, ts in members.items() if topic in ts)
        if not subs:
            continue
        per, extra = divmod(n, len(subs))
        start = 0
        for i, m in enumerate(subs):
            cnt = per + (1 if i < extra else 0)
            if cnt:
                out[m][topic] = list(range(start, start + cnt))
            start += cnt
    return out


class GroupConsumer:
    def __init__(self, client: KafkaClient, topic: str, group_id: str, auto_offset_reset: str = "earliest",
                 session_timeout_ms: int = 10000, max_poll_records: int = 500):
        self.client = client
        self.topic = topic
        self.group = group_id
        self.reset = auto_offset_reset
        self.session_timeout = session_timeout_ms
        self.max_poll = max_poll_records
        self.member_id = ""
        self.generation = -1
        self.assigned: List[int] = []
        self.positions: Dict[int, int] = {}
        self._acked: Dict[int, set] = {}
        self._committed: Dict[int, int] = {}
        self._coord: Optional[KafkaConnection] = None
        self._need_rejoin = True
        self._stop = threading.Event()
        self._hb: Optional[threading.Thread] = None
        self._lock = threading.RLock()
        self._commit_error: Optional[BaseException] = None
        # asynchronous offset commits (the reference's commitAsync, KafkaConsumerWrapper
        # .java:266): commit() records the new contiguous prefix and returns; one committer
        # thread sends the latest offsets per partition, coalescing the calls made while a
        # request was in flight.  flush_commits() sends synchronously (rebalance, close).
        self._pending: Dict[int, int] = {}
        # records fetched beyond max.poll.records, served by the next polls (a fetch
        # response carries up to 1000 records per partition; re-fetching the surplus made
        # the broker encode every record twice)
        self._buf: Dict[int, List[tuple]] = {}
        self._commit_cv = threading.Condition(threading.Lock())
        self._commit_send = threading.Lock()
        self._committer: Optional[threading.Thread] = None

    # -------------------------------------------------------------- membership
    def _coordinator(self) -> KafkaConnection:
        if self._coord is None:
            r = self.client.any_conn().request(P.FIND_COORDINATOR, {"key": self.group})
            if r["error"] != P.NONE:
                raise KafkaError(r["error"], "find coordinator")
            # a dedicated connection: heartbeats must not queue behind long fetches
            self._coord = KafkaConnection(r["host"], r["port"], self.client.client_id)
        return self._coord

    def _join(self) -> None:
        self.flush_commits()   # offsets of the partitions about to be revoked, old generation
        coord = self._coordinator()
        meta = P.encode(P.SUBSCRIPTION, {"version": 0, "topics": [self.topic], "user_data": None})
        while True:
            r = coord.request(P.JOIN_GROUP, {"group_id": self.group, "session_timeout": self.session_timeout,
                                             "rebalance_timeout": self.session_timeout, "member_id": self.member_id,
                                             "protocol_type": "consumer",
                                             "protocols": [{"name": "range", "metadata": meta}]},
                              timeout=self.session_timeout / 1000.0 + 30)
            if r["error"] == P.UNKNOWN_MEMBER_ID:
                self.member_id = ""
                continue
            if r["error"] != P.NONE:
                raise KafkaError(r["error"], "join group")
            break
        self.member_id, self.generation = r["member_id"], r["generation"]
        assignments = []
        if r["leader"] == self.member_id:
            subs = {m["member_id"]: P.decode(P.SUBSCRIPTION, m["metadata"])["topics"] for m in r["members"]}
            parts = {t: self.client.num_partitions(t) for ts in subs.values() for t in ts}
            plan = range_assign(subs, parts)
            for m, tp in plan.items():
                assignments.append({"member_id": m, "assignment": P.encode(P.ASSIGNMENT, {
                    "version": 0, "partitions": [{"topic": t, "partitions": ps} for t, ps in tp.items()],
                    "user_data": None})})
        s = coord.request(P.SYNC_GROUP, {"group_id": self.group, "generation": self.generation,
                                         "member_id": self.member_id, "assignments": assignments},
                          timeout=self.session_timeout / 1000.0 + 30)
        if s["error"] == P.REBALANCE_IN_PROGRESS:
            return  # rejoin on the next poll
        if s["error"] != P.NONE:
            raise KafkaError(s["error"], "sync group")
        a = P.decode(P.ASSIGNMENT, s["assignment"]) if s["assignment"] else {"partitions": []}
        mine = sorted(p for e in a["partitions"] if e["topic"] == self.topic for p in e["partitions"])
        with self._lock:
            self.assigned = mine
            self._init_positions()
            self._need_rejoin = False
        log.info("consumer %s group %s generation %d assigned %s", self.member_id, self.group, self.generation, mine)

    def _init_positions(self) -> None:
        self.positions = {}
        self._buf = {}
        self._acked = {p: set() for p in self.assigned}
        if not self.assigned:
            return
        r = self._coordinator().request(P.OFFSET_FETCH, {"group_id": self.group, "topics": [
            {"name": self.topic, "partitions": self.assigned}]})
        fetched = {p["partition"]: p["offset"] for t in r["topics"] for p in t["partitions"]}
        missing = [p for p in self.assigned if fetched.get(p, -1) < 0]
        defaults = {}
        if missing:
            defaults = self.client.list_offsets(self.topic, -2 if self.reset == "earliest" else -1)
        for p in self.assigned:
            off = fetched.get(p, -1)
            self.positions[p] = off if off >= 0 else defaults.get(p, 0)
            self._committed[p] = self.positions[p]

    def _heartbeat_loop(self) -> None:
        interval = self.session_timeout / 3000.0
        while not self._stop.wait(interval):
            try:
                r = self._coordinator().request(P.HEARTBEAT, {"group_id": self.group, "generation": self.generation,
                                                              "member_id": self.member_id})
                if r["error"] in (P.REBALANCE_IN_PROGRESS, P.ILLEGAL_GENERATION, P.UNKNOWN_MEMBER_ID):
                    self._need_rejoin = True
            except Exception as e:  # noqa: BLE001
                log.debug("heartbeat failed: %s", e)

    def start(self) -> None:
        self._join()
        self._hb = threading.Thread(target=self._heartbeat_loop, daemon=True, name=f"kafka-hb-{self.group}")
        self._hb.start()
        self._committer = threading.Thread(target=self._commit_loop, daemon=True, name=f"kafka-commit-{self.group}")
        self._committer.start()

    def close(self) -> None:
        self._stop.set()
        with self._commit_cv:
            self._commit_cv.notify_all()
        if self._committer is not None:
            self._committer.join(5)
        self.flush_commits()
        try:
            self._coordinator().request(P.LEAVE_GROUP, {"group_id": self.group, "member_id": self.member_id})
        except Exception:  # noqa: BLE001
            pass
        if self._coord is not None:
            self._coord.close()

    # -------------------------------------------------------------- data
    def poll(self, timeout_ms: int = 1000):
        if self._commit_error is not None:
            e, self._commit_error = self._commit_error, None
            raise e
        if self._need_rejoin:
            self._join()
        # max.poll.records caps ONE poll across all partitions (KafkaConsumer semantics);
        # what a fetch returned beyond it waits in _buf, in per-partition order
        with self._lock:
            if any(self._buf.values()):
                out = []
                for p, recs in self._buf.items():
                    room = self.max_poll - len(out)
                    if room <= 0:
                        break
                    out.extend((p,) + r for r in recs[:room])
                    self._buf[p] = recs[room:]
                return out
            pos = dict(self.positions)
        if not pos:
            time.sleep(timeout_ms / 1000.0)
            return []
        res = self.client.fetch(self.topic, pos, max_wait_ms=timeout_ms)
        out = []
        with self._lock:
            for p, (_hw, recs) in res.items():
                if p not in self.positions or self.positions[p] != pos.get(p):
                    continue   # reassigned or moved while the fetch was in flight
                room = max(0, self.max_poll - len(out))
                out.extend((p,) + r for r in recs[:room])
                if len(recs) > room:
                    self._buf[p] = list(recs[room:])
                if recs:
                    self.positions[p] = recs[-1][0] + 1
        return out

    def commit(self, offsets: List[Tuple[int, int]]) -> None:
        """Acknowledge (partition, offset) pairs, possibly out of order; commit the
        contiguous prefix per partition."""
        to_commit = {}
        with self._lock:
            for p, off in offsets:
                if p not in self._acked:
                    continue
                self._acked[p].add(off)
                c = self._committed.get(p, 0)
                s = self._acked[p]
                while c in s:
                    s.discard(c)
                    c += 1
                if c != self._committed.get(p):
                    self._committed[p] = c
                    to_commit[p] = c
        if not to_commit:
            return
        with self._commit_cv:
            self._pending.update(to_commit)
            self._commit_cv.notify()
        if self._committer is None:   # not started (tests driving the consumer directly)
            self.flush_commits()

    def _commit_loop(self) -> None:
        while True:
            with self._commit_cv:
                while not self._pending and not self._stop.is_set():
                    self._commit_cv.wait()
                if self._stop.is_set():
                    return
            self.flush_commits()

    def flush_commits(self) -> None:
        """Send the pending offsets now (synchronous)."""
        with self._commit_send:
            with self._commit_cv:
                batch, self._pending = self._pending, {}
            if not batch:
                return
            try:
                r = self._coordinator().request(P.OFFSET_COMMIT, {
                    "group_id": self.group, "generation": self.generation, "member_id": self.member_id,
                    "retention": -1, "topics": [{"name": self.topic, "partitions": [
                        {"partition": p, "offset": o, "metadata": None} for p, o in sorted(batch.items())]}]})
                for t in r["topics"]:
                    for pr in t["partitions"]:
                        if pr["error"] in (P.REBALANCE_IN_PROGRESS, P.ILLEGAL_GENERATION, P.UNKNOWN_MEMBER_ID):
                            self._need_rejoin = True
                        elif pr["error"] != P.NONE:
                            self._commit_error = KafkaError(pr["error"], "offset commit")
            except Exception as e:  # noqa: BLE001
                self._commit_error = e

    def committed(self) -> Dict[int, int]:
        with self._lock:
            return dict(self._committed)


class PartitionReader:
    def __init__(self, client: KafkaClient, topic: str, start: str = "latest",
                 offsets: Optional[Dict[int, int]] = None):
        self.client = client
        self.topic = topic
        n = client.num_partitions(topic)
        if offsets is not None:
            self.positions = {p: offsets.get(p, 0) for p in range(n)}
        else:
            self.positions = client.list_offsets(topic, -2 if start == "earliest" else -1)

    def read(self, timeout_ms: int = 500):
        res = self.client.fetch(self.topic, dict(self.positions), max_wait_ms=timeout_ms)
        out = []
        for p, (_hw, recs) in sorted(res.items()):
            for r in recs:
                out.append((p,) + r)
            if recs:
                self.positions[p] = recs[-1][0] + 1
        return out
