// Metric data sources of a flow dashboard (datax-metrics metrics.datasource.js, metrics.polling.js,
// metrics.buffer.accumulate.js, metrics.aggregator.js). A flow's `metrics.sources[]` entry names an input
// (MetricApi / MetricDetailsApi / MetricApiRefreshness / Static) and an output shape; the source polls
// /api/metrics/get for new points and publishes dashboard variables named `<source>_<data>` (e.g.
// events_timechart, events_sum) that the widgets bind to.
import { getMetricsData, getMetricsFreshness } from '../common/api.js';

export const aggregators = {
    sum: xs => xs.reduce((a, b) => (isNaN(b) ? a : a + b), 0),
    max: xs => xs.reduce((a, b) => (isNaN(b) ? a : Math.max(a, b)), -Infinity),
    avg: xs => {
        const v = xs.filter(x => !isNaN(x));
        return v.length ? v.reduce((a, b) => a + b, 0) / v.length : NaN;
    }
};

export function normalizeMetricKeys(keys) {
    return (keys || []).map((k, i) => (k && typeof k === 'object' ? k : { name: k, displayName: keys.length > 1 ? 'Shard ' + (i + 1) : String(k) }));
}

// input types -> {series, query(startMs, endMs) -> Promise<per-series point arrays>}
export function makeInput(input, fetchers) {
    const f = fetchers || { get: getMetricsData, freshness: getMetricsFreshness };
    const keys = normalizeMetricKeys(input.metricKeys);
    switch (input.type) {
        case 'MetricApi':
            return {
                series: keys,
                query: (s, e) => Promise.all(keys.map(k => f.get(k.name, s, e).then(rs => rs.map(d => ({ t: +d.uts, v: +d.val })))))
            };
        case 'MetricDetailsApi':
            return {
                series: keys,
                query: (s, e) => Promise.all(keys.map(k => f.get(k.name, s, e).then(rs => rs.map(d => Object.assign({ t: +d.uts, v: +d.val }, d)))))
            };
        case 'MetricApiRefreshness':
            return {
                series: keys,
                query: () => Promise.all(keys.map(k => f.freshness(k.name).then(rs => rs.map(d => ({ t: +d.uts, v: +d.val })))))
            };
        case 'Static':
            return { series: keys.length ? keys : [{ name: 'static', displayName: 'static' }], query: () => Promise.resolve(input.query || []) };
        default:
            throw new Error(`unknown metric input type '${input.type}'`);
    }
}

// Accumulates the points of every series and derives the output variables. `feed(points, nowMs)` takes the new
// points of one poll (per series), returns {var: value} for the variables that changed.
export function makeOutput(output, series, initMs) {
    const want = output.data || {};
    const win = output.chartTimeWindowInMs || 5 * 60 * 1000;
    const hist = series.map(() => []);
    let total = 0;
    let count = 0;
    let first = null;
    const table = series.map(() => []);

    function trim(nowMs) {
        for (const h of hist) while (h.length && h[0].t < nowMs - win) h.shift();
    }

    // events/s between consecutive batches of one series: a batch's count over the gap since the previous batch
    function rates(h) {
        const out = [];
        for (let i = 1; i < h.length; i++) {
            const dt = (h[i].t - h[i - 1].t) / 1000;
            if (dt > 0) out.push([h[i].t, h[i].v / dt]);
        }
        return out;
    }

    function chart(transform) {
        return { series: series.map(s => s.displayName || s.name), x: hist.map(h => transform(h).map(p => p[0])), y: hist.map(h => transform(h).map(p => p[1])) };
    }

    const raw = h => h.map(p => [p.t, p.v]);

    return {
        feed(points, nowMs) {
            const vars = {};
            points.forEach((ps, i) => {
                for (const p of ps) {
                    if (isNaN(p.v) && output.type !== 'DirectTable') continue;
                    hist[i].push(p);
                    if (!isNaN(p.v)) {
                        total += p.v;
                        count += 1;
                    }
                    if (first === null || p.t < first) first = p.t;
                    table[i].push(p);
                    if (table[i].length > 10) table[i].shift();
                }
                hist[i].sort((a, b) => a.t - b.t);
            });
            trim(nowMs);
            const latest = hist.map(h => (h.length ? h[h.length - 1].v : NaN));
            switch (output.type) {
                case 'SumWithTimeChart': {
                    if (want.sum) vars.sum = total;
                    if (want.average) {
                        const minutes = Math.max((nowMs - (first === null ? initMs : Math.min(first, nowMs))) / 60000, 1 / 60);
                        vars.average = total / minutes;
                    }
                    const r = hist.map(h => rates(h));
                    if (want.speed) vars.speed = aggregators.sum(r.map(x => (x.length ? x[x.length - 1][1] : NaN)));
                    if (want.timechart) vars.timechart = chart(rates);
                    break;
                }
                case 'AverageWithTimeChart':
                    if (want.average) vars.average = count ? total / count : NaN;
                    if (want.timechart) vars.timechart = chart(raw);
                    break;
                case 'LatestWithTimeChart':
                    if (want.current) vars.current = aggregators.sum(latest);
                    if (want.timechart) vars.timechart = chart(raw);
                    break;
                case 'SimpleSum':
                    vars.sum = total;
                    break;
                case 'Latest':
                    vars.current = aggregators.max(latest);
                    break;
                case 'DirectTimeChart':
                    if (want.timechart !== false) vars.timechart = chart(raw);
                    if (want.current) vars.current = aggregators.sum(latest);
                    break;
                case 'DirectTable':
                    vars.table = table.map(t => t.slice());
                    break;
                default:
                    throw new Error(`unknown metric output type '${output.type}'`);
            }
            return vars;
        }
    };
}

// One polling data source: start() polls every `pollingInterval` (defaults to the dashboard's) and calls
// onVars({'<name>_<var>': value}); stop() ends it.
export function DataSource(def, onVars, opts) {
    opts = opts || {};
    const input = makeInput(def.input, opts.fetchers);
    const output = def.output || {};
    const now = () => (opts.now ? opts.now() : Date.now());
    let initMs;
    if (output.dynamicOffsetInMs) initMs = now() - output.dynamicOffsetInMs;
    else if (output.type === 'DirectTimeChart' || output.type === 'DirectTable') initMs = now() - (output.chartTimeWindowInMs || 5 * 60 * 1000);
    else {
        const d = new Date(now());
        d.setHours(0, 0, 0, 0);
        initMs = d.getTime();
    }
    const acc = makeOutput(output, input.series, initMs);
    let last = initMs;
    let first = true;
    let timer = null;
    let stopped = false;

    async function poll() {
        const end = now();
        try {
            // scores are server milliseconds and ranges inclusive: the next poll starts one past this one's end
            const pts = await input.query(first ? last : last + 1, end);
            first = false;
            last = end;
            const vars = acc.feed(pts, end);
            const out = {};
            for (const k of Object.keys(vars)) out[`${def.name}_${k}`] = vars[k];
            onVars(out);
        } catch (e) {
            if (opts.onError) opts.onError(e);
        }
    }

    return {
        series: input.series,
        poll,
        start(intervalMs) {
            // the source's own interval, but never slower than the dashboard's refresh
            const every = Math.min((def.input && def.input.pollingInterval) || Infinity, intervalMs || 10000);
            const loop = async () => {
                if (stopped) return;
                await poll();
                if (!stopped) timer = setTimeout(loop, every);
            };
            loop();
        },
        stop() {
            stopped = true;
            if (timer) clearTimeout(timer);
        }
    };
}
