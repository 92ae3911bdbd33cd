"""BASELINE config #5 in miniature (the full 1M-event run is `python -m benchmarks.suite --only 5`):
replay with mid-step connection drops (resume from resourceVersion), bookmarks and
410 compactions (relist + diff), verified exactly-once at the sink."""

import asyncio
import json

from conftest import run
from benchmarks import suite


def test_soak_small_exactly_once():
    class A:
        scale = 0.05

    res = run(suite.config5(A()), timeout=240)
    assert res["duplicates"] == 0
    assert res["drop_only_steps_complete"] is True
    assert res["every_pod_ends_deleted"] is True
    assert res["restarts"] >= 2 and res["compactions_410"] >= 1
    c = res["ours"]["counters"]
    assert c["relists"] >= 2 and c.get("expired_410", 0) >= 1
    assert c["notify_delivered"] == c["notify_submitted"]


def test_replay_server_list_resume_and_410():
    """The replay server behaves like an API server: LIST state, backlog resume, 410."""

    async def body():
        srv = suite.Servers("createdelete", 4)
        async with srv:
            from k8s_watcher_amd.net.http import HttpClient
            c = HttpClient(f"http://127.0.0.1:{srv.api_port}")
            await srv.cmd("PACE 0 0 5")  # first 5 of 12 events, unthrottled
            lst = json.loads((await c.request("GET", "/api/v1/pods")).body)
            rv = int(lst["metadata"]["resourceVersion"])
            live = [i["metadata"]["name"] for i in lst["items"]]
            got = []

            def sink(data, _):
                got.append(data)

            stream, _err = await c.stream("GET", "/api/v1/pods", sink, query={"watch": "true",
                                                                         "resourceVersion": str(rv - 2)})
            await asyncio.sleep(0.2)
            backlog = b"".join(got)
            stream.close()
            await srv.cmd("EXPIRE")
            got.clear()
            stream, _err = await c.stream("GET", "/api/v1/pods", sink, query={"watch": "true",
                                                                         "resourceVersion": str(rv - 2)})
            await asyncio.sleep(0.2)
            expired = b"".join(got)
            stream.close()
            await c.close()
            return rv, live, backlog, expired

    rv, live, backlog, expired = run(body())
    assert rv == 10_000_000 + 4  # five events sent: RVs 10000000..10000004
    assert len(live) == 1  # pod 0 added+modified+deleted, pod 1 added+modified
    lines = [json.loads(l) for l in backlog.splitlines() if l.strip()]
    assert [int(e["object"]["metadata"]["resourceVersion"]) for e in lines] == [rv - 1, rv]
    assert b'"code": 410' in expired or b'"code":410' in expired
