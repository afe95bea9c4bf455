"""Composition demo runtime A: text operations (reference API: apps/composition-demo/runtime_a.py:37-49)."""
import time

from ray import serve


@serve.deployment(ray_actor_options={"num_cpus": 1, "num_gpus": 0, "memory": 512 * 1024**2})
class RuntimeA:
    def __init__(self) -> None:
        self.start = time.time()

    async def test_deployment(self) -> None:
        assert (await self.process_text("a b"))["word_count"] == 2

    async def ping(self) -> str:
        return "pong"

    async def get_status(self) -> dict:
        return {"name": "runtime_a", "status": "ok", "capabilities": ["text_processing"],
                "uptime": time.time() - self.start}

    async def process_text(self, text: str) -> dict:
        words = text.split()
        return {"word_count": len(words), "char_count": len(text), "char_count_no_spaces": len(text.replace(" ", "")),
                "words": words, "reversed": text[::-1], "upper": text.upper(), "lower": text.lower(),
                "title": text.title()}

    async def transform_text(self, text: str) -> dict:
        r = await self.process_text(text)
        return {"upper": r["upper"], "words": r["word_count"]}
