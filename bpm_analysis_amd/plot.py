"""Interactive analysis plot of analyze_wav_file (the plot half).

Restates the reference's ``Plotter`` figure (bpm_analysis.py:429-780): the
decimated envelope and noise floor, trough markers, S1/S2/noise markers with
their formatted decision details as hover text, the BPM curve, belief trend
and HRV traces, slope segments, min/max and summary annotations, the dark
layout with mm:ss ticks.  ``write_plot`` saves ``<base>_bpm_plot.html`` and
returns the figure (what the Gradio app displays).  Parity: the figure's
plotly JSON equals the reference's (tests/test_beats.py::test_plot_matches_reference).
"""
from __future__ import annotations

import datetime
import os
from typing import Dict, List, Optional

import numpy as np
import pandas as pd

from .reports import format_lone_s1_details, format_pairing_details

_HOVER = "%{customdata}<extra></extra>"
_NB4 = "&nbsp;&nbsp;&nbsp;&nbsp;"


def _dt(seconds) -> pd.DatetimeIndex:
    e = datetime.datetime.fromtimestamp(0)
    return pd.to_datetime([e + datetime.timedelta(seconds=t) for t in seconds])


def _peak_hover(p, why: str, sr: int, env) -> str:
    """Hover text of one labelled peak (:570-605)."""
    parts = why.split('§')
    out = [f"<b>Type:</b> {parts[0]}", f"<b>Time:</b> {p / sr:.2f}s", f"<b>Amp:</b> {env[p]:.0f}", "---"]
    rest = parts[1:]
    for i in range(0, len(rest), 2):
        tag, val = rest[i], rest[i + 1] if i + 1 < len(rest) else ""
        if "PAIRING" in tag:
            lines = format_pairing_details(val)
        elif "LONE_S1_REJECT_REASON" in tag or "LONE_S1_VALIDATE_REASON" in tag:
            lines = format_lone_s1_details(val)
        elif "ORIGINAL_REASON" in tag:
            lines = ["- Original Classification:", f"{_NB4}- {val.replace('`', '')}"]
        else:
            lines = []
        if lines:
            out.append("<br>".join(ln.replace('\t', _NB4) for ln in lines))
    return "<br>".join(out)


def _kind(why: str) -> str:
    """'s1' / 's2' / 'noise' from a debug string's leading label (:607-629, PeakType.is_s1/is_s2 :38-46)."""
    label = why.strip()
    if why:
        for sep in ('. Pairing Justification: ', '. Rejection: ', '. Original: ', '. '):
            if sep in why:
                label = why.split(sep, 1)[0].strip()
                break
    else:
        label = "Unknown Peak"
    label = label.strip()
    if label.startswith("S1") or label.startswith("Lone S1"):
        return "s1"
    return "s2" if label.startswith("S2") else "noise"


def build_figure(file_name: str, params: Dict, sr: int, env: np.ndarray, raw_peaks, data: Dict, m: Dict):
    import plotly.graph_objects as go
    from plotly.subplots import make_subplots

    fig = make_subplots(specs=[[{"secondary_y": True}]])
    t_sec = np.arange(len(env)) / sr
    t_dt = _dt(t_sec)

    # envelope + floor, every k-th sample (:510-540)
    k = params.get("plot_downsample_factor", 5)
    floor = data.get('dynamic_noise_floor_series')
    xs, ys, fl = t_dt, env, floor
    if k > 1 and len(env) >= k:
        xs, ys = t_dt[::k], env[::k]
        if floor is not None and not floor.empty:
            fl = floor.iloc[::k]
    fig.add_trace(go.Scatter(x=xs, y=ys, name="Audio Envelope", line=dict(color="#47a5c4")), secondary_y=False)
    if fl is not None and not fl.empty and len(fl) >= len(xs):
        fig.add_trace(go.Scatter(x=xs, y=fl.values, name="Dynamic Noise Floor",
                                 line=dict(color="green", dash="dot", width=1.5),
                                 hovertemplate="Noise Floor: %{y:.2f}<extra></extra>"), secondary_y=False)

    # troughs (:542-559)
    tr = data.get('trough_indices')
    if tr is not None and tr.size > 0:
        fig.add_trace(go.Scatter(x=_dt(tr / sr), y=env[tr], mode='markers', name='Troughs',
                                 marker=dict(color='green', symbol='circle-open', size=6), visible='legendonly'),
                      secondary_y=False)

    # peaks by label, then never-classified raw peaks as noise (:561-670)
    info = data.get('beat_debug_info', {})
    groups: Dict[str, List] = {"s1": ([], []), "s2": ([], []), "noise": ([], [])}
    for p, why in info.items():
        idx, hover = groups[_kind(why)]
        idx.append(p)
        hover.append(_peak_hover(p, why, sr, env))
    for p in raw_peaks:
        if p not in info:
            groups["noise"][0].append(p)
            groups["noise"][1].append(f"<b>Type:</b> Unclassified<br><b>Time:</b> {p / sr:.2f}s<br>"
                                      f"<b>Amp:</b> {env[p]:.0f}<br>"
                                      "<b>Details:</b> Peak was not evaluated by the classifier.")
    for key, name, marker in (("s1", 'S1 Beats', dict(color='#e36f6f', size=8, symbol='diamond')),
                              ("s2", 'S2 Beats', dict(color='orange', symbol='circle', size=6)),
                              ("noise", 'Noise/Rejected', dict(color='grey', symbol='x', size=6))):
        idx, hover = groups[key]
        if idx:
            fig.add_trace(go.Scatter(x=_dt(np.array(idx) / sr), y=env[idx], mode='markers', name=name,
                                     marker=marker, customdata=hover, hovertemplate=_HOVER), secondary_y=False)

    # BPM, belief, HRV (:672-692)
    s = m.get('smoothed_bpm')
    if s is not None and not s.empty:
        fig.add_trace(go.Scatter(x=s.index, y=s.values, name="Average BPM", line=dict(color="#4a4a4a", width=3)),
                      secondary_y=True)
    lt = data.get("long_term_bpm_series")
    if lt is not None and not lt.empty:
        fig.add_trace(go.Scatter(x=_dt(lt.index), y=lt.values, name="BPM Trend (Belief)",
                                 line=dict(color='orange', width=2, dash='dot'), visible='legendonly'),
                      secondary_y=True)
    h = m.get('windowed_hrv_df')
    if h is not None and not h.empty and all(c in h for c in ('time', 'rmssdc', 'sdnn')):
        ht = _dt(h['time'])
        fig.add_trace(go.Scatter(x=ht, y=h['rmssdc'], name="RMSSDc", line=dict(color='cyan', width=2),
                                 visible='legendonly'), secondary_y=True)
        fig.add_trace(go.Scatter(x=ht, y=h['sdnn'], name="SDNN", line=dict(color='magenta', width=2),
                                 visible='legendonly'), secondary_y=True)

    # slope segments (:733-780)
    seg = "<br>Duration: %{customdata[0]:.1f}s<br>BPM {}: %{customdata[1]:.1f}<br>Slope: %{customdata[2]:.2f} BPM/sec<extra></extra>"
    for runs, key, name, color, what in ((m.get('major_inclines'), 'bpm_increase', 'Exertion', "purple", "Increase"),
                                         (m.get('major_declines'), 'bpm_decrease', 'Recovery', "#2ca02c", "Decrease")):
        for i, r in enumerate(runs or []):
            c = [r['duration_sec'], r[key], r['slope_bpm_per_sec']]
            fig.add_trace(go.Scatter(
                x=[r['start_time'], r['end_time']], y=[r['start_bpm'], r['end_bpm']], mode='lines',
                line=dict(color=color, width=4, dash="dash"), name=name, legendgroup=name, showlegend=(i == 0),
                visible='legendonly', yaxis='y2',
                hovertemplate=f"<b>{name} Period</b>" + seg.replace("{}", what), customdata=np.array([c, c])))
    for st, name, color, sign in ((m.get('peak_recovery_stats'), 'Peak Recovery Slope', "#ff69b4", ""),
                                  (m.get('peak_exertion_stats'), 'Peak Exertion Slope', "#9d32a8", "+")):
        if st:
            fig.add_trace(go.Scatter(
                x=[st['start_time'], st['end_time']], y=[st['start_bpm'], st['end_bpm']], mode='lines',
                line=dict(color=color, width=5, dash="solid"), name=name, legendgroup='Steepest Slopes',
                visible='legendonly', yaxis='y2',
                hovertemplate=f"<b>{name}</b><br>Slope: {sign}%{{customdata[0]:.2f}} BPM/sec<br>"
                              "Duration: %{customdata[1]:.1f}s<extra></extra>",
                customdata=np.array([[st['slope_bpm_per_sec'], st['duration_sec']]] * 2)))

    # annotations (:695-731)
    hs, hrr, rec = m.get('hrv_summary'), m.get('hrr_stats'), m.get('peak_recovery_stats')
    if s is not None and not s.empty:
        hi, lo = s.max(), s.min()
        fig.add_annotation(x=s.idxmax(), y=hi, text=f"Max: {hi:.1f} BPM", showarrow=True, arrowhead=1, ax=20,
                           ay=-40, font=dict(color="#e36f6f"), yref="y2")
        fig.add_annotation(x=s.idxmin(), y=lo, text=f"Min: {lo:.1f} BPM", showarrow=True, arrowhead=1, ax=20,
                           ay=40, font=dict(color="#a3d194"), yref="y2")
    if hs:
        txt = "<b>Analysis Summary</b><br>"
        if hs.get('avg_bpm') is not None:
            txt += f"Avg/Min/Max BPM: {hs['avg_bpm']:.1f} / {hs['min_bpm']:.1f} / {hs['max_bpm']:.1f}<br>"
        if hrr and hrr.get('hrr_value_bpm') is not None:
            txt += f"<b>1-Min HRR: {hrr['hrr_value_bpm']:.1f} BPM Drop</b><br>"
        if rec and rec.get('slope_bpm_per_sec') is not None:
            txt += f"<b>Peak Recovery Rate: {rec['slope_bpm_per_sec']:.2f} BPM/sec</b><br>"
        if hs.get('avg_rmssdc') is not None:
            txt += f"Avg. Corrected RMSSD: {hs['avg_rmssdc']:.2f}<br>"
        if hs.get('avg_sdnn') is not None:
            txt += f"Avg. Windowed SDNN: {hs['avg_sdnn']:.2f} ms"
        fig.add_annotation(text=txt, align='left', showarrow=False, xref='paper', yref='paper', x=0.02, y=0.98,
                           bordercolor='black', borderwidth=1, bgcolor='rgba(255, 253, 231, 0.4)')

    # layout (:478-507)
    fig.update_layout(template="plotly_dark", title_text=f"Heartbeat Analysis - {os.path.basename(file_name)}",
                      dragmode='pan', legend=dict(orientation="h", yanchor="bottom", y=1.02, xanchor="right", x=1),
                      margin=dict(t=140, b=100), hovermode='x unified')
    ticks = np.linspace(0, t_sec[-1], num=10)
    e = datetime.datetime.fromtimestamp(0)
    fig.update_xaxes(title_text="Time", tickvals=[e + datetime.timedelta(seconds=x) for x in ticks],
                     ticktext=[f"{int(x // 60):02d}:{int(x % 60):02d} ({x:.2f})" for x in ticks],
                     hoverformat='%M:%S.%L')
    top = np.quantile(fig.data[0].y, 0.95) if fig.data else 1
    fig.update_yaxes(title_text="Signal Amplitude", secondary_y=False,
                     range=[0, top * params.get("plot_amplitude_scale_factor", 60.0)])
    fig.update_yaxes(title_text="BPM / HRV", secondary_y=True, range=[50, 200])
    return fig


def write_plot(file_name: str, output_directory: str, params: Dict, sr: int, env, raw_peaks, data: Dict,
               m: Dict) -> Optional[object]:
    """``<base>_bpm_plot.html`` (:451-456); returns the figure."""
    fig = build_figure(file_name, params, sr, env, raw_peaks, data, m)
    title = f"Heartbeat Analysis - {os.path.basename(file_name)}"
    base = os.path.basename(os.path.splitext(file_name)[0])
    fig.write_html(os.path.join(output_directory, f"{base}_bpm_plot.html"),
                   config={'scrollZoom': True, 'toImageButtonOptions': {'filename': title, 'format': 'png', 'scale': 2}})
    return fig
