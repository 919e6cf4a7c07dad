// Dashboard widgets (datax-metrics components: metricWidgetSimpleBox, metricWidgetPercentageBox,
// metricWidgetNumberBox, metricWidgetGauge / d3.gauge, metricWidgetLineChart, metricWidgetMultiLineChart,
// metricWidgetStackedAreaChart, metricWidgetSimpleTable, metricWidgetDetailsList; dispatch as in
// metricWidgetGeneric.jsx). Charts are inline SVG; no chart library.
import { h, s, formatters, formatTime } from '../common/dom.js';

export const PALETTE = ['#0a68b4', '#e07b00', '#2e9d4f', '#c62828', '#7b4fc9', '#00838f', '#8d6e63', '#d81b60'];

function title(t) {
    return h('div', { class: 'title' }, t);
}

function fmt(name) {
    return formatters[name] || formatters.si;
}

export function SimpleBox(w, value) {
    return h('div', { class: 'widget' }, title(w.displayName), h('div', { class: 'big' }, value === undefined ? '-' : fmt(w.formatter || 'longint')(value)));
}

export function PercentageBox(w, value, base) {
    const pct = base ? value / base : NaN;
    return h('div', { class: 'widget' }, title(w.displayName),
        h('div', { class: 'big' }, value === undefined ? '-' : formatters.longint(value)),
        h('div', { class: 'muted' }, isNaN(pct) ? '-' : formatters.percentage(pct) + ' of ' + formatters.longint(base)));
}

export function Gauge(w, value) {
    const v = value === undefined || isNaN(value) ? 0 : value;
    const max = w.max || Math.max(1, Math.pow(10, Math.ceil(Math.log10(Math.max(v, 1)))));
    const frac = Math.max(0, Math.min(1, v / max));
    const a = Math.PI * (1 - frac);
    const r = 60;
    const arc = (from, to, color) => {
        const x0 = 80 + r * Math.cos(from), y0 = 80 - r * Math.sin(from);
        const x1 = 80 + r * Math.cos(to), y1 = 80 - r * Math.sin(to);
        return s('path', { d: `M ${x0} ${y0} A ${r} ${r} 0 0 1 ${x1} ${y1}`, stroke: color, 'stroke-width': 14, fill: 'none' });
    };
    return h('div', { class: 'widget' }, title(w.displayName),
        s('svg', { viewBox: '0 0 160 100', class: 'gauge', width: '100%', height: '110' },
            arc(Math.PI, 0.0001, '#e3e7ec'),
            frac > 0 ? arc(Math.PI, a + 0.0001, PALETTE[0]) : null,
            s('text', { x: 80, y: 78, 'text-anchor': 'middle', 'font-size': 16 }, formatters.si(v)),
            s('text', { x: 20, y: 96, 'font-size': 9 }, '0'),
            s('text', { x: 140, y: 96, 'text-anchor': 'end', 'font-size': 9 }, formatters.si(max))));
}

// chart data: {series: [names], x: [[ms...] per series], y: [[v...] per series]}
export function chartPaths(data, width, height, opts) {
    opts = opts || {};
    const pad = { l: 44, r: 8, t: 8, b: 18 };
    const xs = [].concat(...data.x);
    if (!xs.length) return null;
    let ys = [].concat(...data.y);
    let stacked = null;
    if (opts.stacked) {
        // align series on the union of times; missing points count as 0
        const times = Array.from(new Set(xs)).sort((a, b) => a - b);
        const acc = times.map(() => 0);
        stacked = data.y.map((yy, i) => {
            const byT = new Map(data.x[i].map((t, j) => [t, yy[j]]));
            const lo = acc.slice();
            times.forEach((t, k) => (acc[k] += byT.get(t) || 0));
            return { times, lo, hi: acc.slice() };
        });
        ys = acc.slice();
    }
    const x0 = Math.min(...xs), x1 = Math.max(...xs);
    const yMax = Math.max(0, ...ys.filter(v => !isNaN(v))) || 1;
    const yMin = opts.stacked ? 0 : Math.min(0, ...ys.filter(v => !isNaN(v)));
    const X = t => pad.l + ((t - x0) / (x1 - x0 || 1)) * (width - pad.l - pad.r);
    const Y = v => height - pad.b - ((v - yMin) / (yMax - yMin || 1)) * (height - pad.t - pad.b);
    const paths = [];
    if (stacked) {
        stacked.forEach((st, i) => {
            const top = st.times.map((t, k) => `${X(t)},${Y(st.hi[k])}`);
            const bot = st.times.map((t, k) => `${X(t)},${Y(st.lo[k])}`).reverse();
            paths.push({ d: `M ${top.join(' L ')} L ${bot.join(' L ')} Z`, color: PALETTE[i % PALETTE.length], fill: true });
        });
    } else {
        data.y.forEach((yy, i) => {
            if (!yy.length) return;
            const pts = yy.map((v, j) => `${X(data.x[i][j])},${Y(v)}`);
            paths.push({ d: 'M ' + pts.join(' L '), color: PALETTE[i % PALETTE.length], fill: false });
        });
    }
    return { paths, x0, x1, yMin, yMax, X, Y, pad };
}

function Chart(w, data, stacked) {
    const W = 600, H = 190;
    const normalizer = w.normalizer === 'percentage' ? v => v * 100 : null;
    if (data && normalizer) data = Object.assign({}, data, { y: data.y.map(yy => yy.map(normalizer)) });
    const geo = data ? chartPaths(data, W, H, { stacked }) : null;
    const body = geo
        ? s('svg', { viewBox: `0 0 ${W} ${H}`, class: 'chart', preserveAspectRatio: 'none' },
            s('line', { class: 'axis', x1: geo.pad.l, y1: H - geo.pad.b, x2: W - geo.pad.r, y2: H - geo.pad.b }),
            s('line', { class: 'axis', x1: geo.pad.l, y1: geo.pad.t, x2: geo.pad.l, y2: H - geo.pad.b }),
            s('text', { x: geo.pad.l - 4, y: geo.pad.t + 8, 'text-anchor': 'end' }, formatters.si(geo.yMax)),
            s('text', { x: geo.pad.l - 4, y: H - geo.pad.b, 'text-anchor': 'end' }, formatters.si(geo.yMin)),
            s('text', { x: geo.pad.l, y: H - 4 }, formatTime(geo.x0)),
            s('text', { x: W - geo.pad.r, y: H - 4, 'text-anchor': 'end' }, formatTime(geo.x1)),
            geo.paths.map(p => s('path', {
                d: p.d,
                stroke: p.color,
                'stroke-width': 1.5,
                fill: p.fill ? p.color : 'none',
                'fill-opacity': p.fill ? 0.35 : null
            })))
        : h('div', { class: 'muted', style: { height: '190px', display: 'flex', alignItems: 'center', justifyContent: 'center' } }, 'No data yet');
    const legend = data && data.series && data.series.length > 1
        ? h('div', { class: 'legend' }, data.series.map((n, i) => h('span', null, h('i', { style: { background: PALETTE[i % PALETTE.length] } }), n)))
        : null;
    return h('div', { class: 'widget' }, title(w.displayName), body, legend);
}

export const LineChart = (w, v) => Chart(w, v, false);
export const MultiLineChart = (w, v) => Chart(w, v, false);
export const StackAreaChart = (w, v) => Chart(w, v, true);

export function SimpleTable(w, value) {
    const rows = Array.isArray(value) ? value : value ? Object.entries(value).map(([k, v]) => ({ name: k, value: v })) : [];
    return h('div', { class: 'widget' }, title(w.displayName),
        h('table', { class: 'grid compact' }, h('tbody', null, rows.map(r => h('tr', null, h('td', null, String(r.name)), h('td', null, String(r.value)))))));
}

// DetailsList: the last rows of an alert source, one table per series (DirectTable output)
export function DetailsList(w, value) {
    const rows = [].concat(...(value || [])).sort((a, b) => b.t - a.t);
    const skip = new Set(['t', 'v']);
    const cols = [];
    for (const r of rows) for (const k of Object.keys(r)) if (!skip.has(k) && !cols.includes(k)) cols.push(k);
    return h('div', { class: 'widget' }, title(w.displayName),
        rows.length
            ? h('table', { class: 'grid compact' },
                h('thead', null, h('tr', null, h('th', null, 'time'), cols.filter(c => c !== 'uts').map(c => h('th', null, c)))),
                h('tbody', null, rows.map(r => h('tr', null, h('td', null, formatTime(r.t)),
                    cols.filter(c => c !== 'uts').map(c => h('td', null, r[c] === undefined ? '' : String(r[c])))))))
            : h('div', { class: 'muted' }, 'No alerts in the window.'));
}

// metricWidgetGeneric.renderWidget: widget config + dashboard variables -> element
export function renderWidget(w, vars) {
    if (!w) return h('div', { class: 'widget' }, 'Null widget');
    if (!w.data) return h('div', { class: 'widget' }, 'Data not configured');
    const value = vars[w.data];
    switch (w.type) {
        case 'SimpleBox':
        case 'NumberBox':
            return SimpleBox(w, value);
        case 'PercentageBox':
            return w.base ? PercentageBox(w, value, vars[w.base]) : h('div', { class: 'widget' }, "'base' parameter is not configured.");
        case 'Gauge':
            return Gauge(w, value);
        case 'LineChart':
            return LineChart(w, value);
        case 'MultiLineChart':
            return MultiLineChart(w, value);
        case 'StackAreaChart':
            return StackAreaChart(w, value);
        case 'SimpleTable':
            return SimpleTable(w, value);
        case 'DetailsList':
            return DetailsList(w, value);
        default:
            return h('div', { class: 'widget' }, `Unknown widget '${w.type}'`);
    }
}
