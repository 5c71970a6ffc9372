"""Store trait (src/io/store/mod.rs:16-45) and the in-memory backend
(src/io/store/memory.rs) used by the reference's own table tests.

RocksDB stays on the host and out of scope; a RocksDB-backed store would
implement the same `read`: look up every key, then feed `add_row` / `add_empty`
in caller order (src/io/store/rocksdb/mod.rs:259-266).
"""
from __future__ import annotations

from dataclasses import dataclass

from .errors import TableAlreadyExists, TableNotFound
from .schema import TableSchema


@dataclass
class KeyValue:
    """src/io/store/mod.rs:16-28."""
    key: bytes
    value: bytes


class Manifest:
    """The part of src/io/store/manifest.rs the store contract needs."""

    def __init__(self):
        self.tables = {}

    def add_table(self, name: str, schema: TableSchema):
        if name in self.tables:
            raise TableAlreadyExists(name)
        self.tables[name] = schema

    def contains(self, name: str) -> bool:
        return name in self.tables

    def schema(self, name: str):
        return self.tables.get(name)


class Store:
    """trait Store (src/io/store/mod.rs:30-45)."""

    def create_table(self, table: str, schema: TableSchema): raise NotImplementedError
    def write(self, table: str, rows): raise NotImplementedError
    def read(self, table: str, keys, builder): raise NotImplementedError
    def compact(self, table: str): raise NotImplementedError
    def manifest(self) -> Manifest: raise NotImplementedError


class MemoryStore(Store):
    """src/io/store/memory.rs:9-64."""

    def __init__(self):
        self.tables = {}
        self._manifest = Manifest()

    def create_table(self, table, schema):
        self._manifest.add_table(table, schema)
        self.tables[table] = {}

    def read(self, table, keys, builder):
        """memory.rs:28-45: Some -> add_row, None -> add_empty, in caller order."""
        rows = self.tables.get(table)
        if rows is None:
            raise TableNotFound(table)
        builder.add_rows([rows.get(bytes(k)) for k in keys])
        return builder.build()

    def write(self, table, rows):
        entries = self.tables.get(table)
        if entries is None:
            raise TableNotFound(table)
        for kv in rows:
            entries[bytes(kv.key)] = bytes(kv.value)

    def compact(self, table):
        return None

    def manifest(self):
        return self._manifest
