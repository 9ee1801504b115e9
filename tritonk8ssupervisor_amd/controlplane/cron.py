"""CronJob schedules: the five-field cron syntax Kubernetes accepts (minute hour day-of-month
month day-of-week; ``*``, lists, ranges, ``/step``, month and weekday names, ``?`` as ``*``),
the ``@yearly/@annually/@monthly/@weekly/@daily/@midnight/@hourly`` macros and ``@every <duration>``
(Go durations such as ``90s``, ``1h30m``; at least one second), plus ``CRON_TZ=``/``TZ=`` prefixes.

As in cron, when both day-of-month and day-of-week are restricted a day matching either runs.
``most_recent(schedule, earliest, now)`` is the controller's question: the latest scheduled time
in (earliest, now], and how many were missed.
"""
from __future__ import annotations

import re
from dataclasses import dataclass
from datetime import datetime, timedelta, timezone

MONTHS = {m: i + 1 for i, m in enumerate("jan feb mar apr may jun jul aug sep oct nov dec".split())}
DAYS = {d: i for i, d in enumerate("sun mon tue wed thu fri sat".split())}
MACROS = {"@yearly": "0 0 1 1 *", "@annually": "0 0 1 1 *", "@monthly": "0 0 1 * *", "@weekly": "0 0 * * 0",
          "@daily": "0 0 * * *", "@midnight": "0 0 * * *", "@hourly": "0 * * * *"}
_DUR = re.compile(r"(\d+(?:\.\d+)?)(h|ms|m|s|us|µs|ns)")
_UNIT = {"h": 3600.0, "m": 60.0, "s": 1.0, "ms": 1e-3, "us": 1e-6, "µs": 1e-6, "ns": 1e-9}


class CronError(ValueError):
    pass


def _field(text: str, lo: int, hi: int, names: dict[str, int] | None = None) -> tuple[frozenset[int], bool]:
    """The values one field allows, and whether it is unrestricted (``*``/``?``)."""
    out: set[int] = set()
    star = False
    for part in text.lower().split(","):
        if not part:
            raise CronError(f"empty list item in {text!r}")
        rng, _, step_s = part.partition("/")
        step = int(step_s) if step_s else 1
        if step_s and (not step_s.isdigit() or step < 1):
            raise CronError(f"bad step in {part!r}")
        if rng in ("*", "?"):
            a, b = lo, hi
            star = star or not step_s
        else:
            a_s, dash, b_s = rng.partition("-")

            def val(s: str) -> int:
                if names and s in names:
                    return names[s]
                if not s.isdigit():
                    raise CronError(f"bad value {s!r} in {text!r}")
                return int(s)

            a = val(a_s)
            b = val(b_s) if dash else (hi if step_s else a)
        if hi == 7 and b == 7:  # day of week 7 is Sunday too
            out.add(0)
            b = 6 if a <= 6 else 7
        if not (lo <= a <= hi and lo <= b <= hi) or a > b:
            raise CronError(f"{part!r} is outside {lo}-{hi}")
        out.update(v % 7 if hi == 7 else v for v in range(a, b + 1, step))
    return frozenset(out), star


def parse_duration(text: str) -> float:
    pos, total = 0, 0.0
    for m in _DUR.finditer(text):
        if m.start() != pos:
            break
        total += float(m.group(1)) * _UNIT[m.group(2)]
        pos = m.end()
    if pos != len(text) or not text:
        raise CronError(f"bad duration {text!r}")
    return total


@dataclass(frozen=True)
class Schedule:
    minutes: frozenset = frozenset()
    hours: frozenset = frozenset()
    dom: frozenset = frozenset()
    months: frozenset = frozenset()
    dow: frozenset = frozenset()
    dom_star: bool = True
    dow_star: bool = True
    every: float = 0.0          # @every: a fixed period in seconds
    tz: timezone | None = None  # None: the control plane's local time

    def _day_ok(self, t: datetime) -> bool:
        d_ok, w_ok = t.day in self.dom, (t.isoweekday() % 7) in self.dow
        if self.dom_star or self.dow_star:
            return d_ok and w_ok
        return d_ok or w_ok

    def next_after(self, t: datetime) -> datetime:
        """The first scheduled time strictly after ``t`` (aware datetime)."""
        if self.every:
            return t + timedelta(seconds=self.every)
        loc = t.astimezone(self.tz) if self.tz else t.astimezone()
        c = (loc + timedelta(minutes=1)).replace(second=0, microsecond=0)
        limit = c + timedelta(days=366 * 5)
        while c < limit:
            if c.month not in self.months:
                c = (c.replace(day=1, hour=0, minute=0) + timedelta(days=32)).replace(day=1)
                continue
            if not self._day_ok(c):
                c = (c + timedelta(days=1)).replace(hour=0, minute=0)
                continue
            if c.hour not in self.hours:
                c = (c + timedelta(hours=1)).replace(minute=0)
                continue
            if c.minute not in self.minutes:
                c += timedelta(minutes=1)
                continue
            return c
        raise CronError("the schedule never fires")


def parse(schedule: str, time_zone: str | None = None) -> Schedule:
    text = schedule.strip()
    tz = None
    m = re.match(r"^(?:CRON_TZ|TZ)=(\S+)\s+(.*)$", text)
    if m:
        time_zone, text = m.group(1), m.group(2)
    if time_zone:
        try:
            from zoneinfo import ZoneInfo

            tz = ZoneInfo(time_zone)
        except Exception as e:  # noqa: BLE001 - any lookup failure is an invalid schedule
            raise CronError(f"unknown time zone {time_zone!r}") from e
    if text.startswith("@every "):
        secs = parse_duration(text[len("@every "):].strip())
        if secs < 1:
            secs = 1.0  # as cron libraries do: sub-second periods run every second
        return Schedule(every=float(round(secs)), tz=tz)
    text = MACROS.get(text.lower(), text)
    parts = text.split()
    if len(parts) != 5:
        raise CronError(f"expected 5 fields (minute hour day-of-month month day-of-week), got {len(parts)}")
    mi, _ = _field(parts[0], 0, 59)
    hr, _ = _field(parts[1], 0, 23)
    dom, dom_star = _field(parts[2], 1, 31)
    mon, _ = _field(parts[3], 1, 12, MONTHS)
    dow, dow_star = _field(parts[4], 0, 7, DAYS)
    return Schedule(mi, hr, dom, mon, dow, dom_star, dow_star, tz=tz)


def most_recent(sched: Schedule, earliest: datetime, now: datetime, cap: int = 100) -> tuple[datetime | None, int]:
    """(latest scheduled time in (earliest, now] or None, number of scheduled times in that
    window, counted up to ``cap``)."""
    t = sched.next_after(earliest)
    if t > now:
        return None, 0
    if sched.every:  # closed form: no need to walk a fast period
        n = int((now - earliest).total_seconds() // sched.every)
        return earliest + timedelta(seconds=n * sched.every), n
    last, n = t, 1
    while n < cap:
        nxt = sched.next_after(last)
        if nxt > now:
            return last, n
        last, n = nxt, n + 1
    # many missed: jump close to now and take the latest from there
    probe = sched.next_after(now - timedelta(days=1)) if now - last > timedelta(days=1) else last
    while (nxt := sched.next_after(probe)) <= now:
        probe = nxt
    return probe, n
