"""model-runner test-report caching and publishing (bioengine_worker_amd/bioimageio/report.py) against
the in-process hub's artifact manager: the reference behaviour of
apps/model-runner/entry_deployment.py:1151-1182, 1573-1819."""
import asyncio
import json

import httpx

from bioengine_worker_amd import __version__
from bioengine_worker_amd.bioimageio import report as rep


def test_env_rows_and_bioengine_row():
    rows = rep.env_rows({"torch": "2.x"})
    names = [r[0] for r in rows]
    assert names[:2] == ["bioimageio.core", "bioimageio.spec"]
    assert ["bioengine", __version__, "", ""] in rows and all(len(r) == 4 for r in rows)
    # an older dict-shaped env is converted; an existing bioengine row is updated in place
    r = rep.ensure_bioengine_row({"env": {"torch": "1"}})
    assert r["env"] == [["torch", "1", "", ""], ["bioengine", __version__, "", ""]]
    r = rep.ensure_bioengine_row({"env": [("bioengine", "0.0.1")]})
    assert r["env"] == [["bioengine", __version__, "", ""]]


def test_cached_report_keyed_on_package_and_versions():
    cur = {"bioimageio.core": "1.0", "bioimageio.spec": "2.0"}
    report = {"status": "passed", "tested_at": 5.0,
              "env": [["bioimageio.core", "1.0", "", ""], ["bioimageio.spec", "2.0", "", ""]]}
    c = {"latest_remote_modified": 42.0, "test_report": report}
    assert rep.cached_report_valid(c, 42.0, cur)
    assert not rep.cached_report_valid(c, 43.0, cur)                      # package changed
    assert not rep.cached_report_valid(c, 42.0, dict(cur, **{"bioimageio.core": "1.1"}))  # impl upgraded
    assert not rep.cached_report_valid({"latest_remote_modified": 42.0, "report": report}, 42.0, cur)  # old layout
    assert not rep.cached_report_valid({"latest_remote_modified": 42.0,
                                        "test_report": {k: v for k, v in report.items() if k != "tested_at"}},
                                       42.0, cur)


def test_publish_report_to_artifact(tmp_path):
    from bioengine_worker_amd.transport.hub import Hub

    async def main():
        hub = Hub(name="report", data_dir=str(tmp_path / "hub"))
        await hub.start_http()
        am = hub.artifacts
        ctx = {"user": {"id": "curator"}, "ws": "bioimage-io"}
        await am.create(type="model", alias="tiny", manifest={"name": "tiny", "test_reports": [{"old": 1}],
                                                              "test_report": {"old": 2}, "score": 0.5},
                        stage=True, context=ctx)
        async with httpx.AsyncClient() as c:
            await c.put(await am.put_file("bioimage-io/tiny", "rdf.yaml", context=ctx), content=b"type: model\n")
            await c.put(await am.put_file("bioimage-io/tiny", rep.LEGACY_REPORT_FILE, context=ctx), content=b"[]")
        await am.commit("bioimage-io/tiny", context=ctx)

        async def http_get(url):
            async with httpx.AsyncClient() as c:
                r = await c.get(url)
                r.raise_for_status()
                return r.text

        puts = []

        async def http_put(url, body):
            puts.append(url)
            async with httpx.AsyncClient() as c:
                (await c.put(url, content=body)).raise_for_status()

        report = rep.finalize_report({"status": "passed", "details": [], "env": rep.env_rows()}, 1234.5)
        assert await rep.publish_report(am, "bioimage-io/tiny", report, http_get, http_put) == "published"
        art = await am.read("bioimage-io/tiny", context=ctx)
        assert not art.get("staging")
        m = art["manifest"]
        assert m["name"] == "tiny" and not ({"test_reports", "test_report", "score"} & set(m))
        assert m["test_summary"] == {"status": "passed", "tested_at": 1234.5, "env": report["env"]}
        names = {f["name"] for f in await am.list_files("bioimage-io/tiny", context=ctx)}
        assert rep.REPORT_FILE in names and rep.LEGACY_REPORT_FILE not in names and "rdf.yaml" in names
        remote = json.loads(await http_get(await am.get_file("bioimage-io/tiny", rep.REPORT_FILE, context=ctx)))
        assert remote == json.loads(json.dumps(report))

        # same tested_at on the artifact: nothing is uploaded again
        assert await rep.publish_report(am, "bioimage-io/tiny", report, http_get, http_put) == "up-to-date"
        assert len(puts) == 1

        # a newer run publishes; an artifact that was staged goes back into staging afterwards
        await am.edit("bioimage-io/tiny", stage=True, context=ctx)
        newer = rep.finalize_report(dict(report, status="failed"), 2000.0)
        assert await rep.publish_report(am, "bioimage-io/tiny", newer, http_get, http_put) == "published"
        art = await am.read("bioimage-io/tiny", context=ctx)
        assert [v["version"] for v in art["versions"]] == ["v0"]
        assert (await am.read("bioimage-io/tiny", version="stage", context=ctx))["staging"]
        committed = await am.read("bioimage-io/tiny", version="v0", context=ctx)
        assert committed["manifest"]["test_summary"]["tested_at"] == 2000.0
        await hub.stop_http()

    asyncio.run(asyncio.wait_for(main(), 60))
