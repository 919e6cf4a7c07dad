"""Design-time and job storage (the reference's CosmosDB / LiteDB ``local.db`` stores:
Services/DataX.Config/DataX.Config.Local/LocalDesignTimeStorage.cs, DataX.Config.Storage/CosmosDBConfigStorage.cs).

* ``DocumentStore`` — SQLite (stdlib) with one table per collection holding JSON documents keyed by name; safe for
  concurrent service threads (one connection per call, WAL mode).  The onebox / single-node default.
* ``CosmosDocumentStore`` — the same interface over a Cosmos DB account (collections ``flows``, ``sparkJobs``,
  ``commons``; document id = name), for a control plane shared by several nodes.
* ``open_store(spec)`` picks one: a path → SQLite; ``cosmos:<connection string>;Database=<db>`` (may be a
  ``keyvault://`` reference) → Cosmos."""
from __future__ import annotations

import json
import os
import sqlite3
import threading
from typing import Any, Dict, List, Optional


class DocumentStore:
    COLLECTIONS = ("flows", "sparkJobs", "commons")

    def __init__(self, path: str):
        self.path = path
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        self._lock = threading.Lock()
        with self._conn() as c:
            c.execute("PRAGMA journal_mode=WAL")
            for coll in self.COLLECTIONS:
                c.execute(f'CREATE TABLE IF NOT EXISTS "{coll}" (name TEXT PRIMARY KEY, doc TEXT NOT NULL)')

    def _conn(self):
        return sqlite3.connect(self.path, timeout=30)

    def upsert(self, coll: str, name: str, doc: Dict[str, Any]):
        with self._lock, self._conn() as c:
            c.execute(f'INSERT INTO "{coll}"(name, doc) VALUES(?, ?) ON CONFLICT(name) DO UPDATE SET doc=excluded.doc',
                      (name, json.dumps(doc)))

    def get(self, coll: str, name: str) -> Optional[Dict[str, Any]]:
        with self._conn() as c:
            row = c.execute(f'SELECT doc FROM "{coll}" WHERE name=?', (name,)).fetchone()
        return json.loads(row[0]) if row else None

    def get_all(self, coll: str) -> List[Dict[str, Any]]:
        with self._conn() as c:
            rows = c.execute(f'SELECT doc FROM "{coll}" ORDER BY name').fetchall()
        return [json.loads(r[0]) for r in rows]

    def delete(self, coll: str, name: str) -> bool:
        with self._lock, self._conn() as c:
            cur = c.execute(f'DELETE FROM "{coll}" WHERE name=?', (name,))
            return cur.rowcount > 0


class CosmosDocumentStore:
    """``DocumentStore`` API over Cosmos DB REST (``dxa.io.azure.CosmosClient``); ids are document names."""
    COLLECTIONS = DocumentStore.COLLECTIONS

    def __init__(self, conn: str, database: str = "production", client=None):
        from ..io.azure import CosmosClient
        self.db = database
        self.client = client or CosmosClient(conn)

    def upsert(self, coll: str, name: str, doc: Dict[str, Any]):
        self.client.upsert(self.db, coll, {**doc, "id": name})

    @staticmethod
    def _strip(d: Optional[Dict[str, Any]]) -> Optional[Dict[str, Any]]:
        if d is None:
            return None
        return {k: v for k, v in d.items() if not k.startswith("_") and k != "id"}

    def get(self, coll: str, name: str) -> Optional[Dict[str, Any]]:
        return self._strip(self.client.get(self.db, coll, name))

    def get_all(self, coll: str) -> List[Dict[str, Any]]:
        docs = sorted(self.client.list(self.db, coll), key=lambda d: d.get("id", ""))
        return [self._strip(d) for d in docs]

    def delete(self, coll: str, name: str) -> bool:
        return self.client.delete(self.db, coll, name)


def open_store(spec: str):
    if spec.startswith("cosmos:"):
        from ..config.secrets import resolve
        conn = resolve(spec[len("cosmos:"):]) or ""
        parts = [p for p in conn.split(";") if p]
        db = next((p.split("=", 1)[1] for p in parts if p.lower().startswith("database=")), "production")
        conn = ";".join(p for p in parts if not p.lower().startswith("database="))
        return CosmosDocumentStore(conn, db)
    return DocumentStore(spec)
