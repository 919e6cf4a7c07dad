"""Design-time and job storage (the reference's CosmosDB / LiteDB ``local.db`` stores:
Services/DataX.Config/DataX.Config.Local/LocalDesignTimeStorage.cs, DataX.Config.Storage/CosmosDBConfigStorage.cs).

SQLite (stdlib) with one table per collection holding JSON documents keyed by name; safe for concurrent service
threads (one connection per call, WAL mode)."""
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
