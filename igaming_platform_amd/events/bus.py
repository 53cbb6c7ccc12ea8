"""In-process domain-event bus (replaces the reference's RabbitMQ library, pkg/events/publisher.go).

Same envelope (``Event``: id, type, source, aggregate_id, timestamp, version, data,
metadata; publisher.go:47-56), the same exchange / routing-key names (publisher.go:17-44)
and the same delivery semantics, without a broker (none exists offline):

* topic exchanges with AMQP-style routing patterns (``*`` one word, ``#`` zero or more);
* queues BOUND to exchanges (the reference declares queues but never binds them, quirk Q17);
* at-least-once delivery to each queue, manual ack: a handler exception nacks and requeues
  (publisher.go:363-371) up to ``max_redeliveries``, then the message goes to the queue's
  dead-letter list; an undecodable payload is rejected without requeue (publisher.go:350-356);
* "publisher confirms" = ``publish`` returns after every bound queue has stored the message.

:class:`RiskEventConsumer` is the feature-update path: wallet transaction
events -> ``RiskEngine.ingest_events`` (K6 on the owner GPU).
"""
from __future__ import annotations

import json
import threading
import time
import uuid
from collections import deque
from dataclasses import asdict, dataclass, field
from typing import Callable, Deque, Dict, List, Optional

from ..obs.logging import get_logger

log = get_logger("events")

# event types (publisher.go:17-32)
ACCOUNT_CREATED = "account.created"
TRANSACTION_COMPLETED = "transaction.completed"
TRANSACTION_FAILED = "transaction.failed"
DEPOSIT_RECEIVED = "deposit.received"
WITHDRAWAL_REQUESTED = "withdrawal.requested"
WITHDRAWAL_COMPLETED = "withdrawal.completed"
BET_PLACED = "bet.placed"
WIN_PAID = "win.paid"
BONUS_AWARDED = "bonus.awarded"
BONUS_COMPLETED = "bonus.completed"
BONUS_EXPIRED = "bonus.expired"
RISK_SCORE_HIGH = "risk.score.high"
RISK_BLOCKED = "risk.blocked"
FRAUD_DETECTED = "fraud.detected"

# exchanges / queues (publisher.go:35-44)
EXCHANGE_WALLET, EXCHANGE_BONUS, EXCHANGE_RISK = "wallet.events", "bonus.events", "risk.events"
QUEUE_RISK_SCORING, QUEUE_BONUS_PROCESSOR = "risk.scoring", "bonus.processor"
QUEUE_ANALYTICS, QUEUE_NOTIFICATIONS = "analytics.events", "notifications.events"


@dataclass
class Event:
    type: str
    source: str
    aggregate_id: str
    data: Dict = field(default_factory=dict)
    id: str = field(default_factory=lambda: str(uuid.uuid4()))
    timestamp: float = field(default_factory=time.time)
    version: int = 1
    metadata: Dict[str, str] = field(default_factory=dict)

    def to_json(self) -> bytes:
        return json.dumps(asdict(self), default=str).encode()

    @classmethod
    def from_json(cls, b: bytes) -> "Event":
        d = json.loads(b)
        return cls(**d)


def topic_match(pattern: str, key: str) -> bool:
    """AMQP topic match: words split on '.', ``*`` = exactly one word, ``#`` = zero or more."""
    p, k = pattern.split("."), key.split(".")

    def m(i: int, j: int) -> bool:
        if i == len(p):
            return j == len(k)
        if p[i] == "#":
            return any(m(i + 1, jj) for jj in range(j, len(k) + 1))
        if j == len(k):
            return False
        return (p[i] == "*" or p[i] == k[j]) and m(i + 1, j + 1)

    return m(0, 0)


@dataclass
class _Msg:
    body: bytes
    routing_key: str
    exchange: str
    redeliveries: int = 0


class Queue:
    def __init__(self, name: str, max_redeliveries: int = 5):
        self.name = name
        self.max_redeliveries = max_redeliveries
        self.msgs: Deque[_Msg] = deque()
        self.dead: List[_Msg] = []
        self.cv = threading.Condition()
        self.acked = 0

    def put(self, m: _Msg) -> None:
        with self.cv:
            self.msgs.append(m)
            self.cv.notify()

    def get(self, timeout: Optional[float] = None) -> Optional[_Msg]:
        with self.cv:
            if not self.msgs:
                self.cv.wait(timeout)
            return self.msgs.popleft() if self.msgs else None

    def __len__(self) -> int:
        return len(self.msgs)


class EventBus:
    def __init__(self):
        self._lock = threading.Lock()
        self.exchanges: Dict[str, List] = {EXCHANGE_WALLET: [], EXCHANGE_BONUS: [], EXCHANGE_RISK: []}
        self.queues: Dict[str, Queue] = {}
        self.published = 0

    def declare_exchange(self, name: str) -> None:
        with self._lock:
            self.exchanges.setdefault(name, [])

    def declare_queue(self, name: str, max_redeliveries: int = 5) -> Queue:
        with self._lock:
            return self.queues.setdefault(name, Queue(name, max_redeliveries))

    def bind(self, queue: str, exchange: str, pattern: str = "#") -> None:
        with self._lock:
            if exchange not in self.exchanges:
                raise KeyError(f"unknown exchange {exchange}")
            q = self.queues[queue]
            self.exchanges[exchange].append((pattern, q))

    def publish(self, exchange: str, event: Event, routing_key: Optional[str] = None) -> int:
        """Persist to every bound queue; returns the number of queues that stored it (the confirm)."""
        key = routing_key or event.type
        body = event.to_json()
        with self._lock:
            if exchange not in self.exchanges:
                raise KeyError(f"unknown exchange {exchange}")
            targets = [q for p, q in self.exchanges[exchange] if topic_match(p, key)]
        for q in {id(q): q for q in targets}.values():
            q.put(_Msg(body, key, exchange))
        self.published += 1
        return len(targets)


class Consumer:
    """Pulls from one queue with manual ack (``prefetch`` messages per loop)."""

    def __init__(self, bus: EventBus, queue: str, handler: Callable[[Event], None], prefetch: int = 10):
        self.q = bus.queues[queue]
        self.handler = handler
        self.prefetch = prefetch
        self._stop = threading.Event()
        self._t: Optional[threading.Thread] = None

    def process_once(self, timeout: float = 0.0) -> int:
        n = 0
        for _ in range(self.prefetch):
            m = self.q.get(timeout if n == 0 else 0)
            if m is None:
                break
            n += 1
            try:
                ev = Event.from_json(m.body)
            except Exception:  # reject, no requeue (publisher.go:350-356)
                log.error("rejecting undecodable message", extra={"fields": dict(queue=self.q.name)})
                self.q.dead.append(m)
                continue
            try:
                self.handler(ev)
                self.q.acked += 1
            except Exception as e:  # nack + requeue (publisher.go:363-371), bounded
                m.redeliveries += 1
                if m.redeliveries > self.q.max_redeliveries:
                    log.error("dead-lettering message", extra={"fields": dict(queue=self.q.name, error=str(e))})
                    self.q.dead.append(m)
                else:
                    self.q.put(m)
        return n

    def start(self) -> "Consumer":
        def loop():
            while not self._stop.is_set():
                self.process_once(timeout=0.1)
        self._t = threading.Thread(target=loop, name=f"consumer-{self.q.name}", daemon=True)
        self._t.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._t is not None:
            self._t.join(timeout=2)


# ---- constructors (publisher.go:397-468)
def transaction_event(event_type: str, tx: Dict) -> Event:
    keys = ("transaction_id", "account_id", "type", "amount", "balance_before", "balance_after", "status",
            "game_id", "round_id", "risk_score")
    return Event(event_type, "wallet-service", str(tx.get("account_id", "")), {k: tx.get(k) for k in keys})


def bonus_event(event_type: str, b: Dict) -> Event:
    keys = ("bonus_id", "account_id", "rule_id", "type", "amount", "wagering_required", "wagering_progress")
    return Event(event_type, "bonus-service", str(b.get("account_id", "")), {k: b.get(k) for k in keys})


def risk_event(event_type: str, account_id: str, score: int, action: str, reasons: List[str]) -> Event:
    return Event(event_type, "risk-service", account_id,
                 {"account_id": account_id, "score": score, "action": action, "reason_codes": reasons})


class RiskEventConsumer:
    """wallet.events -> risk.scoring queue -> RiskEngine.ingest_events (feature updates
    for transactions the engine did not score itself, e.g. wins and refunds)."""

    TYPES = ("win", "refund", "bonus", "bonus_grant")

    def __init__(self, bus: EventBus, engine, batch: int = 256):
        self.engine = engine
        bus.declare_queue(QUEUE_RISK_SCORING)
        bus.bind(QUEUE_RISK_SCORING, EXCHANGE_WALLET, "transaction.#")
        self.consumer = Consumer(bus, QUEUE_RISK_SCORING, self._handle, prefetch=batch)

    def _handle(self, ev: Event) -> None:
        d = ev.data
        if d.get("type") not in self.TYPES or d.get("status") != "completed":
            return
        self.engine.ingest_events([dict(account_id=d["account_id"], amount=int(d["amount"]),
                                        transaction_type="bonus" if d["type"] == "bonus_grant" else d["type"],
                                        ts=int(ev.timestamp))])
