"""``server t``: count the workers that are online (server.go:123-156).

The reference listens for N seconds (default 11) with a 1 s countdown, keeps
every accepted connection, then prints ``####Online Client[n]####`` and one
``[i]Client IP:port[addr]`` line per connection, closes them all and prints a
timestamp.  Workers that connected here receive no job; after the close they
redial (client.go:46-48).  v1 workers also announce ``hello;<id>;<gpu>``, which is
shown next to the address.
"""
from __future__ import annotations

import asyncio
import time

from . import protocol as proto


async def census_async(duration: float = 11, port: int = 8055, host: str = "0.0.0.0", log=print,
                       on_listen=None) -> list[dict]:
    clients: list[dict] = []
    writers = []

    async def on_conn(reader, writer):
        peer = writer.get_extra_info("peername")
        ent = {"addr": f"{peer[0]}:{peer[1]}" if peer else "?", "worker": "", "gpu": ""}
        clients.append(ent)
        writers.append(writer)
        try:
            first = await proto.read_message(reader, timeout=duration)
            line = first.decode(errors="replace").rstrip("\r\n")
            if line.startswith("hello;"):
                parts = line.split(";")
                ent["worker"] = parts[1] if len(parts) > 1 else ""
                ent["gpu"] = parts[2] if len(parts) > 2 else ""
        except (asyncio.TimeoutError, proto.ProtocolError, ConnectionError, OSError):
            pass

    log(f"t:[{int(duration)}]")
    try:
        server = await asyncio.start_server(on_conn, host, port, reuse_address=True)
    except OSError as e:
        log(f"Failure to listen: {e}")
        raise
    if on_listen:
        on_listen(server.sockets[0].getsockname()[1])
    remaining = duration
    while remaining > 0:
        step = min(1.0, remaining)
        await asyncio.sleep(step)
        remaining -= step
        if remaining >= 1:
            log(f"{int(remaining)}")
    server.close()
    log(f"####Online Client[{len(clients)}]####")
    for i, c in enumerate(clients):
        extra = f" {c['worker']} gpu[{c['gpu']}]" if c["worker"] else ""
        log(f"[{i}]Client IP:port[{c['addr']}]{extra}")
    for w in writers:
        w.close()
    log(time.strftime("%Y-%m-%d %H:%M:%S"))
    return clients


def census(duration: float = 11, port: int = 8055, host: str = "0.0.0.0", log=print, on_listen=None) -> list[dict]:
    return asyncio.run(census_async(duration, port, host, log, on_listen))
