"""Synthetic raw datasets with the reference schemas.

The reference's raw archives (``example_data/*.nc``) are not available, so these
generators produce data of the same shape and schema, with physics chosen so that
the spatial context matters (the mechanism the paper's GCN exploits):

* **CML** - microwave links around a centre point. Total loss ``TL_1/TL_2`` =
  per-link baseline + diurnal drift + noise + **rain attenuation** from moving,
  spatially coherent rain cells (seen by every link the cell passes: NOT an
  anomaly) + sensor-specific **anomalies** on the flagged links (jumps, dew bumps,
  fluctuations, unknown drops/spikes) that only that link shows. Four simulated
  experts flag each anomaly with boundary jitter; the label is >=3 experts
  (``create_target``). Gaps and >200 dB spikes emulate data problems.
* **SoilNet** - boxes with sensors at 6 depths; moisture responds to site-wide
  rain with depth-dependent lag and damping, temperature follows a damped diurnal
  cycle, battery voltage decays with recharges. Sensor-specific faults (drops,
  spikes, drift, noise) are flagged ``moisture_flag_Manual``; normal data
  ``moisture_flag_OK``; some periods are unlabelled.
"""
from __future__ import annotations

import numpy as np

from .raw_io import SensorData

_KM_PER_DEG_LAT = 111.2


def _offset_latlon(lat0, lon0, dx_km, dy_km):
    lat = lat0 + dy_km / _KM_PER_DEG_LAT
    lon = lon0 + dx_km / (_KM_PER_DEG_LAT * np.cos(np.radians(lat0)))
    return lat, lon


def _smooth_bump(n, rise, rng):
    """A smooth 0->1->0 envelope of length n."""
    t = np.linspace(0, np.pi, n)
    return np.sin(t) ** (1.0 + rise * rng.random())


def _rain_field(n_sensors, n_time, mx, my, rng, rain_fraction=0.06, minutes_per_step=1.0):
    """Rain rate [sensor, time] (mm/h) from moving Gaussian rain cells."""
    rate = np.zeros((n_sensors, n_time), dtype=np.float32)
    total_h = n_time * minutes_per_step / 60.0
    n_cells = max(1, int(total_h * rain_fraction / 1.5))
    for _ in range(n_cells):
        dur = int(rng.uniform(30, 300) / minutes_per_step)
        t0 = int(rng.integers(0, max(1, n_time - dur)))
        # cell path across the domain
        ang = rng.uniform(0, 2 * np.pi)
        speed = rng.uniform(15, 60) / 60.0 * minutes_per_step  # km per step
        start = np.array([rng.uniform(-25, 25), rng.uniform(-25, 25)])
        radius = rng.uniform(3, 14)
        peak = rng.gamma(2.0, 8.0)
        tt = np.arange(dur)
        cx = start[0] + np.cos(ang) * speed * (tt - dur / 2)
        cy = start[1] + np.sin(ang) * speed * (tt - dur / 2)
        env = _smooth_bump(dur, 1.0, rng)
        # small-scale variability within the cell
        env = env * np.clip(1 + 0.3 * np.convolve(rng.standard_normal(dur), np.ones(9) / 9, "same"), 0.2, 2)
        d2 = (mx[:, None] - cx[None, :]) ** 2 + (my[:, None] - cy[None, :]) ** 2
        rate[:, t0:t0 + dur] += (peak * env[None, :] * np.exp(-d2 / (2 * radius ** 2))).astype(np.float32)
    return rate


def _rainlike_attenuation(rng, T, kcoef1, kcoef2, length):
    """(t0, prof1, prof2): the attenuation a rain cell passing over ONE link would cause (a cell drawn
    like :func:`_rain_field`'s - duration, peak, small-scale variability - with its track through the
    link, seen by no other link), through the same power law and wet-antenna term as real rain."""
    dur = int(rng.uniform(30, 300))
    t0 = int(rng.integers(0, max(1, T - dur)))
    speed = rng.uniform(15, 60) / 60.0
    radius = rng.uniform(3, 14)
    miss = rng.uniform(0, 0.7) * radius                 # closest approach of the track to the link
    peak = rng.gamma(2.0, 8.0)
    tt = np.arange(dur)
    along = speed * (tt - dur * rng.uniform(0.3, 0.7))
    env = _smooth_bump(dur, 1.0, rng)
    env = env * np.clip(1 + 0.3 * np.convolve(rng.standard_normal(dur), np.ones(9) / 9, "same"), 0.2, 2)
    rate = peak * env * np.exp(-(along ** 2 + miss ** 2) / (2 * radius ** 2))
    wet = 1.2 * (1 - np.exp(-rate / 1.5))
    return t0, kcoef1 * rate ** 1.05 * length + wet, kcoef2 * rate ** 1.05 * length + wet


def _inject_cml_anomalies(rng, tl1, tl2, flags, flag_names, s, T, days, anomaly_rate, difficulty, n_exp,
                          rainlike_frac=0.0, link=None):
    """Anomaly events of flagged link ``s`` added to its TL rows, with the experts' flags.

    ``rainlike_frac`` > 0: that fraction of the events is rain-shaped (:func:`_rainlike_attenuation`,
    flagged as ``Dew``: a wet antenna without rain). On the link's own series such an event is drawn
    from the same distribution as real rain attenuation; only the neighbours tell them apart (real
    rain cells are seen by every link they pass). ``link`` = (kcoef1, kcoef2,
    length) of link ``s``."""
    n_events = rng.poisson(anomaly_rate * days * 1.6)
    base_p = np.array([0.3, 0.25, 0.3, 0.15])
    for _ in range(n_events):
        if rainlike_frac > 0:
            kind = rng.choice(5, p=list(base_p * (1.0 - rainlike_frac)) + [rainlike_frac])
        else:
            kind = rng.choice(4, p=base_p)
        if kind == 4:    # rain-like: a wet-antenna event with rain's rise and decay
            t0, p1, p2 = _rainlike_attenuation(rng, T, *link)
            dur = len(p1)
            tl1[s, t0:t0 + dur] += p1
            tl2[s, t0:t0 + dur] += p2
            on = np.nonzero(p1 > 0.1 * max(float(p1.max()), 1e-6))[0]
            a0, a1 = t0 + int(on[0]), t0 + int(on[-1]) + 1
            for e in range(n_exp):
                if rng.random() < 0.92:
                    j0 = int(np.clip(a0 + rng.integers(-6, 7), 0, T - 1))
                    j1 = int(np.clip(a1 + rng.integers(-6, 7), j0 + 1, T))
                    flags[flag_names[1]][e, s, j0:j1] = True
            continue
        if kind == 0:    # jump: level shift for a while
            dur = int(rng.uniform(20, 240))
            t0 = int(rng.integers(0, T - dur))
            amp = rng.choice([-1, 1]) * rng.uniform(1.0, 6.0) / difficulty
            prof = np.ones(dur) * amp
            ramp = min(3, dur // 4)
            if ramp > 0:
                prof[:ramp] *= np.linspace(0.3, 1, ramp)
        elif kind == 1:  # dew: morning bump
            dur = int(rng.uniform(60, 240))
            day0 = int(rng.integers(0, max(1, int(days) - 1)))
            t0 = min(T - dur - 1, day0 * 1440 + int(rng.uniform(180, 420)))
            amp = rng.uniform(1.0, 4.0) / difficulty
            prof = amp * _smooth_bump(dur, 0.5, rng)
        elif kind == 2:  # fluctuation: high-frequency noise burst
            dur = int(rng.uniform(30, 240))
            t0 = int(rng.integers(0, T - dur))
            sig = rng.uniform(0.6, 2.5) / difficulty
            prof = rng.normal(0, sig, dur) + np.abs(rng.normal(0, sig / 2, dur))
        else:            # unknown: deep drops/spikes or drift
            dur = int(rng.uniform(10, 120))
            t0 = int(rng.integers(0, T - dur))
            amp = rng.uniform(3, 12) / difficulty
            prof = amp * (rng.random(dur) < 0.3) * rng.uniform(0.3, 1.0, dur)
        tl1[s, t0:t0 + dur] += prof
        tl2[s, t0:t0 + dur] += prof * rng.uniform(0.7, 1.1)
        name = flag_names[kind]
        for e in range(n_exp):
            if rng.random() < 0.92:
                j0 = int(np.clip(t0 + rng.integers(-6, 7), 0, T - 1))
                j1 = int(np.clip(t0 + dur + rng.integers(-6, 7), j0 + 1, T))
                flags[name][e, s, j0:j1] = True


def make_cml_raw(n_sensors: int = 23, n_flagged: int = 1, n_minutes: int = 40320,
                 start: str = "2019-07-02T00:00", seed: int = 0, center=(51.5, 7.45),
                 extent_km: float = 12.0, anomaly_rate: float = 1.0, rain_fraction: float = 0.06,
                 gap_rate: float = 2e-4, difficulty: float = 1.0, rainlike_frac: float = 0.0) -> SensorData:
    """CML raw dataset (schema of ``cml_raw_example.nc``).

    ``anomaly_rate`` scales the number of anomaly events per flagged link
    (1.0 ~ 10-15% anomalous minutes); ``difficulty`` scales how rain-like the
    anomalies look (amplitudes/shape overlap with rain attenuation).
    ``rainlike_frac``: fraction of the anomaly events that are rain-shaped wet-antenna events seen by
    the flagged link only (:func:`_rainlike_attenuation`): on the link's own series they cannot be
    told from rain, so only the neighbourhood separates them (0 = none; the RNG stream is then the
    one of earlier versions).
    """
    rng = np.random.default_rng(seed)
    S, T = n_sensors, n_minutes
    time = np.arange(np.datetime64(start, "m"), np.datetime64(start, "m") + np.timedelta64(T, "m"))
    # --- geometry: link mid-points in a disc, random orientation and length
    r = extent_km * np.sqrt(rng.random(S))
    th = rng.uniform(0, 2 * np.pi, S)
    mx, my = r * np.cos(th), r * np.sin(th)
    length = rng.uniform(0.5, 12.0, S)
    orient = rng.uniform(0, np.pi, S)
    ax_, ay_ = mx - np.cos(orient) * length / 2, my - np.sin(orient) * length / 2
    bx_, by_ = mx + np.cos(orient) * length / 2, my + np.sin(orient) * length / 2
    lat_a, lon_a = _offset_latlon(center[0], center[1], ax_, ay_)
    lat_b, lon_b = _offset_latlon(center[0], center[1], bx_, by_)
    freq1 = rng.choice([15.0, 18.0, 23.0, 26.0, 32.0, 38.0], S)
    freq2 = freq1 + rng.choice([-1.0, 1.0], S) * rng.uniform(0.5, 1.5, S)
    pol1 = rng.choice(np.array(["H", "V"]), S)
    pol2 = np.where(rng.random(S) < 0.8, pol1, np.where(pol1 == "H", "V", "H"))
    # --- baseline signal
    minute_of_day = (np.arange(T) % 1440).astype(np.float32)
    diurnal = np.sin(2 * np.pi * (minute_of_day - 300) / 1440.0)
    base1 = rng.uniform(40, 70, S)[:, None]
    base2 = base1 + rng.normal(0, 2.0, S)[:, None]
    drift_amp = rng.uniform(0.1, 0.5, S)[:, None]
    slow = np.cumsum(rng.normal(0, 0.01, (S, T)), axis=1).astype(np.float32)
    slow -= np.linspace(0, 1, T)[None, :] * slow[:, -1:]
    tl1 = base1 + drift_amp * diurnal[None, :] + slow + rng.normal(0, 0.12, (S, T))
    tl2 = base2 + drift_amp * 0.9 * diurnal[None, :] + slow + rng.normal(0, 0.12, (S, T))
    # --- rain attenuation (spatially coherent, not an anomaly)
    rain = _rain_field(S, T, mx, my, rng, rain_fraction=rain_fraction)
    kcoef1 = (0.0009 * freq1 ** 1.8)[:, None]
    kcoef2 = (0.0009 * freq2 ** 1.8)[:, None]
    wet = 1.2 * (1 - np.exp(-rain / 1.5))
    tl1 = tl1 + kcoef1 * rain ** 1.05 * length[:, None] + wet
    tl2 = tl2 + kcoef2 * rain ** 1.05 * length[:, None] + wet
    # --- anomalies on flagged links + expert flags
    flagged = np.zeros(S, bool)
    # flagged links are drawn among the most central links so they have neighbours
    order = np.argsort(mx ** 2 + my ** 2)
    flagged[order[:n_flagged]] = True
    n_exp = 4
    flag_names = ["Jump", "Dew", "Fluctuation", "Unknown anomaly"]
    flags = {k: np.zeros((n_exp, S, T), dtype=bool) for k in flag_names}
    days = T / 1440.0
    for s in np.nonzero(flagged)[0]:
        _inject_cml_anomalies(rng, tl1, tl2, flags, flag_names, s, T, days, anomaly_rate, difficulty, n_exp,
                              rainlike_frac, (float(kcoef1[s, 0]), float(kcoef2[s, 0]), float(length[s])))
    # --- quantisation, gaps, out-of-range spikes
    tl1 = np.round(tl1 * 10) / 10
    tl2 = np.round(tl2 * 10) / 10
    for arr in (tl1, tl2):
        g = rng.random((S, T)) < gap_rate
        for s, t in zip(*np.nonzero(g)):
            arr[s, t:t + int(rng.integers(1, 8))] = np.nan
        spikes = rng.random((S, T)) < gap_rate / 4
        arr[spikes] = 255.0
    # occasional long outages on unflagged links
    for s in range(S):
        if not flagged[s] and rng.random() < 0.3:
            t0 = int(rng.integers(0, T - 600))
            d = int(rng.uniform(60, 600))
            tl1[s, t0:t0 + d] = np.nan
            tl2[s, t0:t0 + d] = np.nan
    ids = np.array([f"SY{1000 + i:04d}_2_SY{5000 + 7 * i:04d}_{1 + i % 4}" for i in range(S)])
    ds = SensorData(attrs={"title": "synthetic CML raw dataset (gnnqc)", "seed": seed})
    ds.set_coord("sensor_id", "sensor_id", ids)
    ds.set_coord("time", "time", time)
    ds.set_coord("expert", "expert", np.arange(n_exp, dtype=np.int32))
    ds.set_coord("length", "sensor_id", length.astype(np.float64))
    ds.set_coord("site_a_latitude", "sensor_id", lat_a)
    ds.set_coord("site_a_longitude", "sensor_id", lon_a)
    ds.set_coord("site_b_latitude", "sensor_id", lat_b)
    ds.set_coord("site_b_longitude", "sensor_id", lon_b)
    ds.set_coord("frequency_1", "sensor_id", freq1)
    ds.set_coord("frequency_2", "sensor_id", freq2)
    ds.set_coord("polarization_1", "sensor_id", pol1)
    ds.set_coord("polarization_2", "sensor_id", pol2)
    ds["TL_1"] = (("sensor_id", "time"), tl1.astype(np.float32))
    ds["TL_2"] = (("sensor_id", "time"), tl2.astype(np.float32))
    for k in flag_names:
        ds[k] = (("expert", "sensor_id", "time"), flags[k])
    ds["flagged"] = ("sensor_id", flagged)
    return ds


def make_cml_raw_network(n_sensors: int = 3904, n_flagged: int = 20, n_minutes: int = 133920,
                         start: str = "2019-07-01T00:00", seed: int = 0, center=(51.16, 10.45),
                         extent_km: float = 337.0, anomaly_rate: float = 1.0, rain_fraction: float = 0.06,
                         gap_rate: float = 2e-4, difficulty: float = 1.0, block: int = 128,
                         min_neighbours: int = 3, max_sample_distance: float = 20.0) -> SensorData:
    """Country-scale CML raw dataset: the full reference network's SHAPE (3,904 links x 133,920
    minutes, 20 flagged links; ``notebooks/prepare_raw_cml.ipynb`` cell 9) with the physics of
    :func:`make_cml_raw`, generated memory-lean: float32 TL rows built in blocks of ``block``
    links, rain cells spread over the whole disc (count scaled with its area) and evaluated only on
    the links near each cell's path, expert flags allocated as zero pages that are written only
    for the flagged links. The default disc (337 km radius ~ Germany's area) gives a 20 km
    neighbourhood of ~14 links, like the real network's density. Flagged links are drawn among
    links with at least ``min_neighbours`` others within ``max_sample_distance`` km."""
    rng = np.random.default_rng(seed)
    S, T = n_sensors, n_minutes
    time = np.arange(np.datetime64(start, "m"), np.datetime64(start, "m") + np.timedelta64(T, "m"))
    r = extent_km * np.sqrt(rng.random(S))
    th = rng.uniform(0, 2 * np.pi, S)
    mx, my = r * np.cos(th), r * np.sin(th)
    length = rng.uniform(0.5, 12.0, S)
    orient = rng.uniform(0, np.pi, S)
    ax_, ay_ = mx - np.cos(orient) * length / 2, my - np.sin(orient) * length / 2
    bx_, by_ = mx + np.cos(orient) * length / 2, my + np.sin(orient) * length / 2
    lat_a, lon_a = _offset_latlon(center[0], center[1], ax_, ay_)
    lat_b, lon_b = _offset_latlon(center[0], center[1], bx_, by_)
    freq1 = rng.choice([15.0, 18.0, 23.0, 26.0, 32.0, 38.0], S)
    freq2 = freq1 + rng.choice([-1.0, 1.0], S) * rng.uniform(0.5, 1.5, S)
    pol1 = rng.choice(np.array(["H", "V"]), S)
    pol2 = np.where(rng.random(S) < 0.8, pol1, np.where(pol1 == "H", "V", "H"))
    # --- rain rate [S, T] float32 from moving cells, each touching only the links near its path
    rain = np.zeros((S, T), dtype=np.float32)
    total_h = T / 60.0
    n_cells = max(1, int(total_h * rain_fraction / 1.5 * (extent_km / 25.0) ** 2))
    for _ in range(n_cells):
        dur = int(rng.uniform(30, 300))
        t0 = int(rng.integers(0, max(1, T - dur)))
        ang = rng.uniform(0, 2 * np.pi)
        speed = rng.uniform(15, 60) / 60.0
        rr = extent_km * np.sqrt(rng.random())
        tt_ = rng.uniform(0, 2 * np.pi)
        start_xy = np.array([rr * np.cos(tt_), rr * np.sin(tt_)])
        radius = rng.uniform(3, 14)
        peak = rng.gamma(2.0, 8.0)
        tt = np.arange(dur)
        cx = start_xy[0] + np.cos(ang) * speed * (tt - dur / 2)
        cy = start_xy[1] + np.sin(ang) * speed * (tt - dur / 2)
        env = _smooth_bump(dur, 1.0, rng)
        env = env * np.clip(1 + 0.3 * np.convolve(rng.standard_normal(dur), np.ones(9) / 9, "same"), 0.2, 2)
        reach = 4.0 * radius
        near = np.nonzero((mx >= cx.min() - reach) & (mx <= cx.max() + reach) &
                          (my >= cy.min() - reach) & (my <= cy.max() + reach))[0]
        if near.size == 0:
            continue
        d2 = (mx[near, None] - cx[None, :]) ** 2 + (my[near, None] - cy[None, :]) ** 2
        rain[near, t0:t0 + dur] += (peak * env[None, :] * np.exp(-d2 / (2 * radius ** 2))).astype(np.float32)
    # --- flagged links: random links with enough neighbours
    cand = []
    for s in rng.permutation(S):
        d = np.hypot(mx - mx[s], my - my[s])
        if int((d <= max_sample_distance).sum()) - 1 >= min_neighbours:
            cand.append(int(s))
            if len(cand) == n_flagged:
                break
    flagged = np.zeros(S, bool)
    flagged[cand] = True
    n_exp = 4
    flag_names = ["Jump", "Dew", "Fluctuation", "Unknown anomaly"]
    flags = {k: np.zeros((n_exp, S, T), dtype=bool) for k in flag_names}     # zero pages until written
    tl1 = np.empty((S, T), dtype=np.float32)
    tl2 = np.empty((S, T), dtype=np.float32)
    minute_of_day = (np.arange(T) % 1440).astype(np.float32)
    diurnal = np.sin(2 * np.pi * (minute_of_day - 300) / 1440.0).astype(np.float32)
    ramp = np.linspace(0, 1, T, dtype=np.float32)
    days = T / 1440.0
    for b0 in range(0, S, block):
        b1 = min(S, b0 + block)
        n = b1 - b0
        br = np.random.default_rng([seed, b0])
        base1 = br.uniform(40, 70, n).astype(np.float32)[:, None]
        base2 = base1 + br.normal(0, 2.0, n).astype(np.float32)[:, None]
        drift_amp = br.uniform(0.1, 0.5, n).astype(np.float32)[:, None]
        slow = np.cumsum(br.normal(0, 0.01, (n, T)).astype(np.float32), axis=1)
        slow -= ramp[None, :] * slow[:, -1:]
        kc1 = (0.0009 * freq1[b0:b1] ** 1.8).astype(np.float32)[:, None]
        kc2 = (0.0009 * freq2[b0:b1] ** 1.8).astype(np.float32)[:, None]
        rb = rain[b0:b1]
        wet = 1.2 * (1 - np.exp(-rb / 1.5))
        att = rb ** 1.05 * length[b0:b1, None].astype(np.float32)
        tl1[b0:b1] = base1 + drift_amp * diurnal[None, :] + slow + br.normal(0, 0.12, (n, T)).astype(np.float32) \
            + kc1 * att + wet
        tl2[b0:b1] = base2 + drift_amp * 0.9 * diurnal[None, :] + slow + \
            br.normal(0, 0.12, (n, T)).astype(np.float32) + kc2 * att + wet
    del rain
    for s in np.nonzero(flagged)[0]:
        _inject_cml_anomalies(rng, tl1, tl2, flags, flag_names, s, T, days, anomaly_rate, difficulty, n_exp)
    for b0 in range(0, S, block):
        b1 = min(S, b0 + block)
        br = np.random.default_rng([seed, b0, 1])
        for arr in (tl1, tl2):
            blk = arr[b0:b1]
            np.round(blk * 10, out=blk)
            blk /= 10
            g = br.random(blk.shape, dtype=np.float32) < gap_rate
            for s_, t_ in zip(*np.nonzero(g)):
                blk[s_, t_:t_ + int(br.integers(1, 8))] = np.nan
            blk[br.random(blk.shape, dtype=np.float32) < gap_rate / 4] = 255.0
    for s in range(S):
        if not flagged[s] and rng.random() < 0.3:
            t0 = int(rng.integers(0, T - 600))
            d = int(rng.uniform(60, 600))
            tl1[s, t0:t0 + d] = np.nan
            tl2[s, t0:t0 + d] = np.nan
    ids = np.array([f"SY{1000 + i:05d}_2_SY{50000 + 7 * i:06d}_{1 + i % 4}" for i in range(S)])
    ds = SensorData(attrs={"title": "synthetic country-scale CML raw dataset (gnnqc)", "seed": seed})
    ds.set_coord("sensor_id", "sensor_id", ids)
    ds.set_coord("time", "time", time)
    ds.set_coord("expert", "expert", np.arange(n_exp, dtype=np.int32))
    ds.set_coord("length", "sensor_id", length.astype(np.float64))
    ds.set_coord("site_a_latitude", "sensor_id", lat_a)
    ds.set_coord("site_a_longitude", "sensor_id", lon_a)
    ds.set_coord("site_b_latitude", "sensor_id", lat_b)
    ds.set_coord("site_b_longitude", "sensor_id", lon_b)
    ds.set_coord("frequency_1", "sensor_id", freq1)
    ds.set_coord("frequency_2", "sensor_id", freq2)
    ds.set_coord("polarization_1", "sensor_id", pol1)
    ds.set_coord("polarization_2", "sensor_id", pol2)
    ds["TL_1"] = (("sensor_id", "time"), tl1)
    ds["TL_2"] = (("sensor_id", "time"), tl2)
    for k in flag_names:
        ds[k] = (("expert", "sensor_id", "time"), flags[k])
    ds["flagged"] = ("sensor_id", flagged)
    return ds


def make_soilnet_raw(n_boxes: int = 40, n_time: int = 8545, start: str = "2014-08-01T00:00",
                     seed: int = 0, center=(51.35, 12.43), extent_m: float = 60.0,
                     fault_rate: float = 1.0, max_sensors: int | None = 210,
                     spatial_fault_frac: float = 0.5) -> SensorData:
    """SoilNet raw dataset (schema of ``soilnet_raw_example.nc``), 15-min resolution.

    Faults are of two families. Self-evident ones (drop, spikes, drift, noise) a model sees in
    the sensor's own series. A ``spatial_fault_frac`` share is only visible against the
    neighbours - the mechanism the reference's GCN exploits (README: GCN 0.858 > baseline
    0.816): a *missed wetting* (the sensor stays on its dry-down while the same-depth sensors
    of its box cluster respond to a rain event) and a *phantom wetting* (an infiltration-shaped
    rise with no rain at the site). Both stay inside the sensor's own plausible range and
    dynamics."""
    rng = np.random.default_rng(seed)
    depths_all = np.array([0.05, 0.1, 0.2, 0.3, 0.4, 0.6])
    box_xy = rng.uniform(-extent_m, extent_m, (n_boxes, 2)) / 1000.0  # km
    # many boxes share one of a few clusters so same-depth neighbours exist within 20 m
    n_clusters = max(1, n_boxes // 4)
    cl = rng.uniform(-extent_m, extent_m, (n_clusters, 2)) / 1000.0
    which = rng.integers(0, n_clusters, n_boxes)
    box_xy = cl[which] + rng.normal(0, 0.008, (n_boxes, 2))
    sensors = []
    for b in range(n_boxes):
        nlev = 6 if rng.random() < 0.75 else int(rng.integers(3, 6))
        for lvl in range(nlev):
            sensors.append((b, lvl, depths_all[lvl]))
    if max_sensors is not None:
        sensors = sensors[:max_sensors]
    S, T = len(sensors), n_time
    box_id = np.array([s[0] for s in sensors], dtype=np.int32)
    level_id = np.array([s[1] for s in sensors], dtype=np.int32)
    depth = np.array([s[2] for s in sensors], dtype=np.float64)
    lat, lon = _offset_latlon(center[0], center[1], box_xy[box_id, 0], box_xy[box_id, 1])
    step_h = 0.25
    tt = np.arange(T)
    hour = (tt * step_h) % 24
    # --- site rain (event based), spatially varying intensity per box
    rain = np.zeros(T)
    n_ev = int(T * step_h / 24 * 0.35)
    for _ in range(n_ev):
        t0 = int(rng.integers(0, max(1, T - 40)))
        d = int(rng.integers(2, 24))
        rain[t0:t0 + d] += rng.gamma(1.5, 1.2)
    box_gain = rng.uniform(0.7, 1.3, n_boxes)[box_id]
    # infiltration: first order response, lag & damping grow with depth
    moist = np.zeros((S, T))
    base = rng.uniform(12, 35, S)
    tau_dry = 150 + 400 * depth  # steps
    for i in range(S):
        lag = int(depth[i] * 40)
        resp = np.convolve(rain, np.exp(-np.arange(200) / (4 + 30 * depth[i])), "full")[:T]
        resp = np.roll(resp, lag)
        resp[:lag] = 0
        from scipy.signal import lfilter
        a = np.exp(-1.0 / tau_dry[i])
        gain = box_gain[i] * (1.6 - depth[i]) * 0.9
        wet = lfilter([1.0], [1.0, -a], gain * resp * 0.12)
        moist[i] = base[i] + np.minimum(wet, 25) + rng.normal(0, 0.15, T)
    # --- temperature
    season = 15 - 8 * (tt / T)
    temp = np.zeros((S, T))
    for i in range(S):
        amp = 8 * np.exp(-depth[i] / 0.12)
        ph = depth[i] * 10
        temp[i] = season + amp * np.sin(2 * np.pi * (hour - 9 - ph) / 24) + rng.normal(0, 0.1, T)
    # --- battery (per box)
    batt_box = np.zeros((n_boxes, T))
    for b in range(n_boxes):
        v = rng.uniform(3300, 3550)
        for t in range(T):
            v -= rng.uniform(0.0, 0.08)
            if v < 2950 and rng.random() < 0.02:
                v = rng.uniform(3400, 3550)
            batt_box[b, t] = v
    battv = batt_box[box_id] + rng.normal(0, 2, (S, T))
    # --- faults (sensor specific) -> manual flags
    manual = np.zeros((S, T), bool)
    n_days = T * step_h / 24
    rain_starts = np.nonzero((rain[1:] > 0.5) & (rain[:-1] <= 0.5))[0] + 1
    rain_c = np.convolve(rain, np.ones(96), "full")[:T]          # rain in the last 24 h
    dry = np.nonzero(rain_c < 1e-6)[0]
    for i in range(S):
        n_f = rng.poisson(fault_rate * n_days / 12)
        for _ in range(n_f):
            kind = rng.integers(0, 4)
            d = int(rng.integers(8, max(9, min(300, T // 2))))
            t0 = int(rng.integers(0, T - d))
            if rng.random() < spatial_fault_frac:
                lag = int(depth[i] * 40)
                if rng.random() < 0.5 and len(rain_starts):
                    # missed wetting: from just before a rain event on, the sensor keeps drying
                    # down (its own recession rate) while its neighbours respond
                    t0 = int(rng.choice(rain_starts)) + lag
                    d = int(min(T - t0, rng.integers(96, 300))) if t0 < T - 8 else 0
                    if d < 8:
                        continue
                    v0 = moist[i, max(t0 - 1, 0)]
                    rec = np.exp(-np.arange(d) / tau_dry[i])
                    moist[i, t0:t0 + d] = base[i] + (v0 - base[i]) * rec + rng.normal(0, 0.15, d)
                elif len(dry) > 0:
                    # phantom wetting: an infiltration-shaped rise without rain at the site
                    t0 = int(rng.choice(dry))
                    d = int(min(T - t0, rng.integers(96, 300)))
                    if d < 8:
                        continue
                    k = np.exp(-np.arange(d) / (4 + 30 * depth[i]))
                    pulse = np.convolve(np.r_[rng.gamma(1.5, 1.2) * np.ones(int(rng.integers(4, 16))),
                                              np.zeros(d)], k, "full")[:d]
                    a = np.exp(-1.0 / tau_dry[i])
                    from scipy.signal import lfilter
                    wet = lfilter([1.0], [1.0, -a], box_gain[i] * (1.6 - depth[i]) * 0.9 * pulse * 0.12)
                    moist[i, t0:t0 + d] = np.minimum(moist[i, t0:t0 + d] + wet, base[i] + 25)
                else:
                    continue
                manual[i, t0:t0 + d] = True
                continue
            if kind == 0:    # drop to implausibly low value
                moist[i, t0:t0 + d] = moist[i, t0:t0 + d] * rng.uniform(0.2, 0.6)
            elif kind == 1:  # spikes
                idx = t0 + np.nonzero(rng.random(d) < 0.3)[0]
                moist[i, idx] += rng.uniform(5, 25, idx.size)
            elif kind == 2:  # drift
                moist[i, t0:t0 + d] += np.linspace(0, rng.uniform(-10, 10), d)
            else:            # noise
                moist[i, t0:t0 + d] += rng.normal(0, rng.uniform(1, 4), d)
            manual[i, t0:t0 + d] = True
    # --- flags
    flags = {}
    no_label = np.zeros((S, T), bool)
    for i in range(S):
        if rng.random() < 0.2:
            d = int(rng.integers(min(50, T // 4), max(min(50, T // 4) + 1, min(800, T // 2))))
            t0 = int(rng.integers(0, T - d))
            no_label[i, t0:t0 + d] = True
    no_label &= ~manual
    auto_batt = battv < 2900
    auto_range = (moist <= 0) | (moist >= 100)
    dm = np.abs(np.diff(moist, axis=1, prepend=moist[:, :1]))
    auto_spike = dm > 8
    ok = ~(manual | no_label | auto_batt | auto_range)
    for var in ("moisture", "temp"):
        flags[f"{var}_flag_no_label"] = no_label.copy()
        flags[f"{var}_flag_Auto:BattV"] = auto_batt.copy()
        flags[f"{var}_flag_Auto:Range"] = auto_range.copy() if var == "moisture" else np.zeros_like(ok)
        flags[f"{var}_flag_Auto:Spike"] = auto_spike.copy() if var == "moisture" else np.zeros_like(ok)
        flags[f"{var}_flag_Manual"] = manual.copy() if var == "moisture" else np.zeros_like(ok)
        flags[f"{var}_flag_OK"] = ok.copy() if var == "moisture" else ~no_label
    # --- gaps
    for arr in (moist, temp, battv):
        g = rng.random((S, T)) < 3e-4
        for i, t in zip(*np.nonzero(g)):
            arr[i, t:t + int(rng.integers(1, 10))] = np.nan
    time = np.arange(np.datetime64(start, "m"), np.datetime64(start, "m") + np.timedelta64(15 * T, "m"),
                     np.timedelta64(15, "m"))
    ds = SensorData(attrs={"title": "synthetic SoilNet raw dataset (gnnqc)", "seed": seed})
    ds.set_coord("sensor_id", "sensor_id", np.arange(S, dtype=np.int64))
    ds.set_coord("time", "time", time)
    ds.set_coord("box_id", "sensor_id", box_id)
    ds.set_coord("level_id", "sensor_id", level_id)
    ds.set_coord("latitude", "sensor_id", lat)
    ds.set_coord("longitude", "sensor_id", lon)
    ds.set_coord("depth", "sensor_id", depth)
    ds["moisture"] = (("sensor_id", "time"), moist.astype(np.float32))
    ds["temp"] = (("sensor_id", "time"), temp.astype(np.float32))
    ds["battv"] = (("sensor_id", "time"), battv.astype(np.float32))
    for k, v in flags.items():
        ds[k] = (("sensor_id", "time"), v)
    return ds


__all__ = ["make_cml_raw", "make_cml_raw_network", "make_soilnet_raw"]
