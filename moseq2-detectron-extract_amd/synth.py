"""Seeded synthetic depth sessions: int16 512x424 Kinect-style
frames of one elliptical "mouse" on a tilted floor plane.

Frames are a pure function of (seed, frame index) so any shard of a session
can be regenerated independently on its own GPU without a 434 GB file.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass

import numpy as np

WIDTH, HEIGHT = 512, 424


@dataclass
class SynthConfig:
    width: int = WIDTH
    height: int = HEIGHT
    floor_mm: float = 670.0
    noise_mm: float = 1.5
    invalid_p: float = 0.002     # Bernoulli rate of Kinect-invalid (0) pixels
    semi_major: float = 40.0     # px
    semi_minor: float = 18.0     # px (>= 13 so clean_frames' 3x opening keeps the body)
    dome_min: float = 15.0       # mm above floor
    dome_max: float = 45.0
    tail_len: float = 25.0
    arena_radius: float = 150.0


def background(cfg: SynthConfig = SynthConfig()) -> np.ndarray:
    yy, xx = np.mgrid[0:cfg.height, 0:cfg.width]
    return (cfg.floor_mm + 0.02 * xx - 0.01 * yy)


def trajectory(n: int, seed: int = 0, cfg: SynthConfig = SynthConfig()):
    """Smoothed random walk of the centre inside the arena; heading follows
    velocity.  Returns centres (n,2) float64 (x, y) and headings (n,) rad."""
    rng = np.random.default_rng(seed)
    cx0, cy0 = cfg.width / 2, cfg.height / 2
    steps = rng.normal(0, 1.0, size=(n + 8, 2))
    k = np.ones(9) / 9.0
    sm = np.stack([np.convolve(steps[:, i], k, mode="valid")[:n] for i in range(2)], 1) * 2.5
    pos = np.empty((n, 2))
    p = np.array([cx0, cy0])
    for i in range(n):
        p = p + sm[i]
        d = p - [cx0, cy0]
        r = np.hypot(*d)
        if r > cfg.arena_radius:
            p = np.array([cx0, cy0]) + d * (cfg.arena_radius / r)
        pos[i] = p
    vel = np.gradient(pos, axis=0)
    head = np.arctan2(vel[:, 1], vel[:, 0] + 1e-9)
    return pos, head


def render(idx: np.ndarray, pos: np.ndarray, head: np.ndarray, seed: int = 0,
           cfg: SynthConfig = SynthConfig()) -> np.ndarray:
    """Render frames `idx` (absolute frame numbers) -> int16 (len(idx), H, W).
    The animal's height is evaluated only inside the square around its centre
    that holds the body and tail (outside it the height is exactly 0), so a
    frame costs its two noise draws plus a small patch."""
    bg = background(cfg)
    yy, xx = np.mgrid[0:cfg.height, 0:cfg.width].astype(np.float64)
    reach = int(np.ceil(np.hypot(cfg.semi_major + cfg.tail_len, max(cfg.semi_minor, 1.0)))) + 2
    out = np.empty((len(idx), cfg.height, cfg.width), np.int16)
    for o, i in enumerate(idx):
        rng = np.random.default_rng([seed, int(i)])
        cx, cy = pos[o]
        th = head[o]
        c, s = np.cos(th), np.sin(th)
        y0, y1 = max(0, int(np.floor(cy)) - reach), min(cfg.height, int(np.floor(cy)) + reach + 1)
        x0, x1 = max(0, int(np.floor(cx)) - reach), min(cfg.width, int(np.floor(cx)) + reach + 1)
        height = np.zeros(bg.shape)
        if y0 < y1 and x0 < x1:
            px, py = xx[y0:y1, x0:x1], yy[y0:y1, x0:x1]
            u = (px - cx) * c + (py - cy) * s
            v = -(px - cx) * s + (py - cy) * c
            r2 = (u / cfg.semi_major) ** 2 + (v / cfg.semi_minor) ** 2
            h = np.where(r2 <= 1, cfg.dome_min + (cfg.dome_max - cfg.dome_min) * np.sqrt(np.clip(1 - r2, 0, 1)), 0)
            tail = (u < -cfg.semi_major) & (u > -cfg.semi_major - cfg.tail_len) & (np.abs(v) <= 1.0)
            height[y0:y1, x0:x1] = np.where(tail, 8.0, h)
        depth = bg - height + rng.normal(0, cfg.noise_mm, size=bg.shape)
        d = np.round(depth).astype(np.int16)
        if cfg.invalid_p > 0:
            d[rng.random(bg.shape) < cfg.invalid_p] = 0
        out[o] = d
    return out


def _render_to_file(args):
    """Process-pool worker of SyntheticSession.write: frames [a, b) into the
    memory-mapped depth.dat."""
    path, nframes, a, b, pos, head, seed, cfg = args
    mm = np.memmap(path, dtype="<i2", mode="r+", shape=(nframes, cfg.height, cfg.width))
    for s in range(a, b, 100):
        e = min(s + 100, b)
        mm[s:e] = render(np.arange(s, e), pos[s - a:e - a], head[s - a:e - a], seed, cfg)
    mm.flush()
    return b - a


class SyntheticSession:
    """In-memory stand-in for M/io/session.py Session: background, roi,
    true_depth and frame chunks (int16 (n,424,512))."""

    def __init__(self, nframes: int, seed: int = 0, cfg: SynthConfig = SynthConfig(), roi: str = "full"):
        self.nframes, self.seed, self.cfg = nframes, seed, cfg
        self.pos, self.head = trajectory(nframes, seed, cfg)
        # background as the reference computes it: median of frames -> .5-granular
        self.bground_im = np.round(background(cfg) * 2) / 2
        if roi == "full":
            self.roi = np.ones((cfg.height, cfg.width), bool)
        else:
            yy, xx = np.mgrid[0:cfg.height, 0:cfg.width]
            self.roi = (xx - cfg.width / 2) ** 2 + (yy - cfg.height / 2) ** 2 <= (cfg.arena_radius + 60) ** 2
        self.true_depth = float(np.median(self.bground_im))
        self.timestamps = np.arange(nframes) * 33.333

    def frames(self, start: int, stop: int) -> np.ndarray:
        idx = np.arange(start, stop)
        return render(idx, self.pos[start:stop], self.head[start:stop], self.seed, self.cfg)

    def iterate(self, chunk_size: int = 1000):
        for s in range(0, self.nframes, chunk_size):
            e = min(s + chunk_size, self.nframes)
            yield np.arange(s, e), self.frames(s, e)

    def write(self, dirname: str, workers: int = 0):
        """Write depth.dat (<i2), metadata.json, depth_ts.txt like a real session.
        workers > 1 renders blocks of frames in that many processes (frames are
        a pure function of (seed, index), so the file is the same)."""
        os.makedirs(dirname, exist_ok=True)
        path = os.path.join(dirname, "depth.dat")
        n = self.nframes
        if workers > 1 and n > 200:
            with open(path, "wb") as fh:
                fh.truncate(n * self.cfg.height * self.cfg.width * 2)
            step = -(-n // workers)
            jobs = [(path, n, a, min(a + step, n), self.pos[a:a + step], self.head[a:a + step], self.seed, self.cfg)
                    for a in range(0, n, step)]
            import concurrent.futures as cf
            import multiprocessing as mp
            import sys
            # spawned, not forked: callers may already hold a HIP context (its
            # runtime threads and device mappings must not be duplicated); the
            # workers only need numpy and this module, registered under its
            # package name by mdx_pkg.load (the repository root is on sys.path)
            root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
            if root not in sys.path:
                sys.path.insert(0, root)
            import mdx_pkg
            with cf.ProcessPoolExecutor(max_workers=len(jobs), mp_context=mp.get_context("spawn"),
                                        initializer=mdx_pkg.load) as ex:
                assert sum(ex.map(_render_to_file, jobs)) == n
        else:
            with open(path, "wb") as fh:
                for _, ch in self.iterate(500):
                    fh.write(ch.astype("<i2").tobytes())
        with open(os.path.join(dirname, "metadata.json"), "w") as fh:
            json.dump({"DepthResolution": [self.cfg.width, self.cfg.height], "SubjectName": "synthetic",
                       "SessionName": f"seed{self.seed}"}, fh)
        np.savetxt(os.path.join(dirname, "depth_ts.txt"), self.timestamps, fmt="%.3f")
