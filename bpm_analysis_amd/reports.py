"""Text reports of analyze_wav_file (the plot is plot.py).

Restates the reference's ``ReportGenerator`` (bpm_analysis.py:782-985) and the
two detail formatters it borrows from ``Plotter`` (:336-427):

* ``<base>_Analysis_Settings.json``  {'start_bpm_hint': ...}            :790-799
* ``<base>_Analysis_Summary.md``     summary, slopes, changes, BPM table :801-813, :908-985
* ``<base>_Debug_Log.md``            one entry per labelled peak / trough :815-906

Same bytes as the reference except the one "generated on" timestamp line of
each markdown file (``now`` is injectable for tests).  The interactive plot
is plot.py.
"""
from __future__ import annotations

import datetime
import json
import logging
import os
import re
from typing import Dict, List, Optional

import numpy as np
import pandas as pd


def _now(now):
    return (now or datetime.datetime.now()).strftime('%Y-%m-%d %H:%M:%S')


# ---------------------------------------------------------------- detail formatters
_NUM_END = re.compile(r'([\d\.]+)$')
_X_NUM = re.compile(r'x([\d\.]+)')
_BY_NUM = re.compile(r'by ([\d\.]+)')


def format_pairing_details(details: str) -> List[str]:
    """A pairing reason -> bullet lines with the running confidence (:336-365)."""
    lines = [ln.strip().lstrip('- ') for ln in details.strip().split('\n') if ln.strip()]
    head = "- S1-S2 pairing decision:"
    if not lines:
        return [head, "    - No details available."]
    try:
        m = _NUM_END.search(lines[0])
        conf = float(m.group(1)) if m else 0.0
        out = [head, f"    - {lines[0]}"]
        for ln in lines[1:]:
            if "Stability Pre-Adjust" in ln:
                m = _X_NUM.search(ln)
                conf *= float(m.group(1)) if m else 1
                out.append(f"    - {ln} -> {conf:.3f}")
            elif "PENALIZED by" in ln or "Interval PENALTY by" in ln:
                m = _BY_NUM.search(ln)
                conf -= float(m.group(1)) if m else 0
                shown = max(0, conf) if "Interval PENALTY by" in ln else conf
                out.append(f"    - {ln} -> {shown:.3f}")
            else:
                out.append(f"    - {ln}")
        return out
    except (ValueError, IndexError):
        return [head, f"    - {details}"]


_LONE = re.compile(r"(Validated|Rejected) Lone S1: Confidence ([\d\.]+) (>=|<) Threshold ([\d\.]+)\. \((.*)\)")
_LONE_PARTS = dict(rf=r"Rhythm Fit=([\d\.]+)", rd=r"\(Interval .*?s vs Expected .*?s\)",
                   af=r"Amplitude Fit=([\d\.]+)", ad=r"\(Strength Ratio .*?x\)",
                   rw=r"Rhythm=([\d\.]+)", aw=r"Amplitude=([\d\.]+)")


def format_lone_s1_details(details: str) -> List[str]:
    """A lone-S1 validation reason -> bullet lines with the weighted sum (:367-427)."""
    head = "- Lone S1 decision:"
    m = _LONE.search(details)
    if not m:
        return [head, f"\t- {details}"]
    try:
        status, conf_s, op, thr_s, why = m.groups()
        conf, thr = float(conf_s), float(thr_s)
        x = {k: re.search(p, why) for k, p in _LONE_PARTS.items()}
        rs, af = float(x['rf'].group(1)), float(x['af'].group(1))
        out = [head, f"\t- Rhythm Fit={rs:.2f} {x['rd'].group(0)}", f"\t- Amplitude Fit={af:.2f} {x['ad'].group(0)}"]
        if x['rw'] and x['aw']:
            rw, aw = float(x['rw'].group(1)), float(x['aw'].group(1))
            out += ["\t- Weighted Calculation:",
                    f"\t\t- Rhythm: {rs:.2f} × {rw:.2f} = {rs * rw:.3f}",
                    f"\t\t- Amplitude: {af:.2f} × {aw:.2f} = {af * aw:.3f}",
                    f"\t\t- Final: {rs * rw:.3f} + {af * aw:.3f} = {conf:.3f}"]
        out.append(f"- Final Score: Confidence {conf:.3f} {op} {thr:.2f} -> "
                   f"{'Validated' if 'Validated' in status else 'Rejected'}")
        return out
    except (AttributeError, ValueError, IndexError) as e:
        logging.warning(f"Could not parse Lone S1 details string: '{details}'. Error: {e}")
        return [head, f"\t- {details}"]


# ---------------------------------------------------------------- files
def _base(file_name: str) -> str:
    return os.path.basename(os.path.splitext(file_name)[0])


def write_settings(file_name: str, output_directory: str, start_bpm_hint: Optional[float]) -> str:
    path = os.path.join(output_directory, f"{_base(file_name)}_Analysis_Settings.json")
    with open(path, "w", encoding="utf-8") as f:
        json.dump({'start_bpm_hint': start_bpm_hint}, f, indent=4)
    return path


def summary_text(file_name: str, m: Dict, now=None) -> str:
    """The Analysis_Summary.md body (:908-985)."""
    w = [f"# Analysis Report for: {os.path.basename(file_name)}\n", f"*Generated on: {_now(now)}*\n\n",
         "## Overall Summary\n\n| Metric | Value |\n|:---|:---|\n"]
    hs, hrr = m.get('hrv_summary'), m.get('hrr_stats')
    if hs:
        if hs.get('avg_bpm') is not None:
            w.append(f"| **Average BPM** | {hs['avg_bpm']:.1f} BPM |\n")
            w.append(f"| **BPM Range** | {hs['min_bpm']:.1f} to {hs['max_bpm']:.1f} BPM |\n")
        if hs.get('avg_rmssdc') is not None:
            w.append(f"| **Avg. Corrected RMSSD** | {hs['avg_rmssdc']:.2f} |\n")
        if hs.get('avg_sdnn') is not None:
            w.append(f"| **Avg. Windowed SDNN** | {hs['avg_sdnn']:.2f} ms |\n")
    if hrr and hrr.get('hrr_value_bpm') is not None:
        w.append(f"| **1-Minute HRR** | {hrr['hrr_value_bpm']:.1f} BPM Drop |\n")
    w.append("\n## Steepest Slopes Analysis\n\n### Peak Exertion (Fastest HR Increase)\n\n")
    for st, sign, none_msg in ((m.get('peak_exertion_stats'), "+", "*No significant peak exertion period found.*"),
                               (m.get('peak_recovery_stats'), "",
                                "*No significant peak recovery period found post-peak.*")):
        if st:
            w.append("| Attribute | Value |\n|:---|:---|\n")
            w.append(f"| **Rate** | `{sign}{st['slope_bpm_per_sec']:.2f}` BPM/second |\n")
            w.append(f"| **Period** | {st['start_time'].strftime('%M:%S')} to {st['end_time'].strftime('%M:%S')} |\n")
            w.append(f"| **Duration** | {st['duration_sec']:.1f} seconds |\n")
            w.append(f"| **BPM Change** | {st['start_bpm']:.1f} to {st['end_bpm']:.1f} BPM |\n\n")
        else:
            w.append(none_msg + "\n\n")
        if sign == "+":
            w.append("### Peak Recovery (Fastest HR Decrease)\n\n")
    w.append("## All Significant HR Changes\n\n### Exertion Periods (Sustained HR Increase)\n\n")
    epoch = datetime.datetime.fromtimestamp(0)
    for runs, key, sign, title in ((m.get('major_inclines'), 'bpm_increase', "+", None),
                                   (m.get('major_declines'), 'bpm_decrease', "-",
                                    "\n### Recovery Periods (Sustained HR Decrease)\n\n")):
        if title:
            w.append(title)
        if runs:
            for r in runs:
                a = (r['start_time'] - epoch).total_seconds()
                b = (r['end_time'] - epoch).total_seconds()
                w.append(f"- **From {a:.1f}s to {b:.1f}s:** Duration={r['duration_sec']:.1f}s, "
                         f"Change=`{sign}{r[key]:.1f}` BPM\n")
        else:
            w.append("*None found.*\n")
    w.append("\n## Heartbeat Data (BPM over Time)\n\n| Time (s) | Average BPM |\n|:---:|:---:|\n")
    s, t = m.get('smoothed_bpm'), m.get('bpm_times')
    if s is not None and not s.empty and t is not None:
        w.extend(f"| {x:.2f} | {b:.1f} |\n" for x, b in zip(t, s.values) if not np.isnan(b))
    else:
        w.append("| *No data* | *No data* |\n")
    return "".join(w)


def _log_frame(env, sr, raw_peaks, data: Dict, s: Optional[pd.Series], t) -> Optional[pd.DataFrame]:
    """Peak/trough events joined to the nearest (<= 0.5 s) floor / BPM / belief values (:827-855)."""
    info = data.get('beat_debug_info', {})
    ev = [{'time': p / sr, 'type': 'Peak', 'amp': env[p], 'reason': info.get(p)} for p in raw_peaks if info.get(p)]
    if 'trough_indices' in data:
        ev += [{'time': p / sr, 'type': 'Trough', 'amp': env[p], 'reason': ''} for p in data['trough_indices']]
    if not ev:
        return None
    events = pd.DataFrame(ev).sort_values(by='time').set_index('time')
    grid = pd.DataFrame(index=np.arange(len(env)) / sr)
    if 'dynamic_noise_floor_series' in data:
        grid['noise_floor'] = data['dynamic_noise_floor_series'].values
    if s is not None and not s.empty:
        grid['smoothed_bpm'] = pd.Series(data=s.values, index=t).groupby(level=0).mean()
    lt = data.get('long_term_bpm_series')
    if lt is not None and not lt.empty:
        grid['lt_bpm'] = lt.groupby(level=0).mean()
    grid.ffill(inplace=True)
    return pd.merge_asof(left=events, right=grid, left_index=True, right_index=True, direction='nearest',
                         tolerance=0.5)


_DETAIL = (("PAIRING", format_pairing_details), ("LONE_S1_REJECT_REASON", format_lone_s1_details),
           ("LONE_S1_VALIDATE_REASON", format_lone_s1_details))
_LOG_METRICS = (("Raw Amp", 'amp'), ("Noise Floor", 'noise_floor'), ("Average BPM (Smoothed)", 'smoothed_bpm'),
                ("Long-Term BPM (Belief)", 'lt_bpm'))


def debug_log_text(file_name: str, env, sr, raw_peaks, data: Dict, m: Dict, now=None) -> str:
    """The Debug_Log.md body (:815-906)."""
    df = _log_frame(env, sr, raw_peaks, data, m.get('smoothed_bpm'), m.get('bpm_times'))
    if df is None or df.empty:
        return "# No significant events detected to log.\n"
    w = [f"# Chronological Debug Log for {os.path.basename(file_name)}\n", f"Analysis performed on: {_now(now)}\n\n"]
    cols = set(df.columns)
    for row in df.itertuples(name="LogEvent"):
        w.append(f"## Time: `{row.Index:.4f}s`\n")
        if row.type == 'Trough':
            w.append("**Trough Detected**\n")
        else:
            why = getattr(row, 'reason', '')
            if not why or why == 'Unknown':
                w.append("**Unclassified Peak**\n")
            else:
                parts = why.split('§')
                w.append(f"**{parts[0]}.**\n")
                rest = parts[1:]
                for i in range(0, len(rest), 2):
                    tag, val = rest[i], rest[i + 1] if i + 1 < len(rest) else ""
                    lines = None
                    for key, fmt in _DETAIL:
                        if key in tag:
                            lines = "\n".join(fmt(val))
                            break
                    if lines is None and "ORIGINAL_REASON" in tag:
                        lines = f"- Original Classification:\n    - `{val}`"
                    if lines:
                        w.append(f"{lines}\n")
        for name, col in _LOG_METRICS:
            v = getattr(row, col) if col in cols else None
            if pd.notna(v):
                w.append(f"- **{name}**: `{v:.1f}`\n")
        w.append("\n\n")
    return "".join(w)


def write_reports(file_name: str, output_directory: str, env, sr, raw_peaks, data: Dict, m: Dict,
                  start_bpm_hint: Optional[float], now=None) -> None:
    """Summary, debug log and settings, as analyze_wav_file writes them (:1762-1765)."""
    b = _base(file_name)
    with open(os.path.join(output_directory, f"{b}_Analysis_Summary.md"), "w", encoding="utf-8") as f:
        f.write(summary_text(file_name, m, now))
    with open(os.path.join(output_directory, f"{b}_Debug_Log.md"), "w", encoding="utf-8") as f:
        f.write(debug_log_text(file_name, env, sr, raw_peaks, data, m, now))
    write_settings(file_name, output_directory, start_bpm_hint)
