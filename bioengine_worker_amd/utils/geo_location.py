"""Worker geo-location (reference: bioengine/utils/geo_location.py:19-157).

Tries a chain of public IP-geolocation services; returns ``None`` fields when offline (the worker
reports whatever it could resolve in ``get_status()['geo_location']``)."""
from __future__ import annotations

import httpx

_PROVIDERS = (
    ("https://ipwho.is/", lambda d: (d.get("city"), d.get("region"), d.get("country"), d.get("latitude"), d.get("longitude"))),
    ("http://ip-api.com/json/", lambda d: (d.get("city"), d.get("regionName"), d.get("country"), d.get("lat"), d.get("lon"))),
    ("https://ipapi.co/json/", lambda d: (d.get("city"), d.get("region"), d.get("country_name"), d.get("latitude"), d.get("longitude"))),
)


async def fetch_geolocation(timeout: float = 3.0) -> dict:
    async with httpx.AsyncClient(timeout=timeout) as c:
        for url, parse in _PROVIDERS:
            try:
                r = await c.get(url)
                if r.status_code != 200:
                    continue
                city, region, country, lat, lon = parse(r.json())
                if country:
                    return {"city": city, "region": region, "country": country, "latitude": lat, "longitude": lon}
            except Exception:
                continue
    return {"city": None, "region": None, "country": None, "latitude": None, "longitude": None}


async def fetch_centroid_coordinates(query: str, timeout: float = 3.0):
    try:
        async with httpx.AsyncClient(timeout=timeout, headers={"User-Agent": "bioengine-worker-amd"}) as c:
            r = await c.get("https://nominatim.openstreetmap.org/search", params={"q": query, "format": "json", "limit": 1})
            js = r.json()
            if js:
                return float(js[0]["lat"]), float(js[0]["lon"])
    except Exception:
        pass
    return None
