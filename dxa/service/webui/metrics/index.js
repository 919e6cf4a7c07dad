// Metric explorer (datax-metrics components/metricExplorer.jsx, metricDashboard.jsx, metricAllProducts.jsx): a flow
// list on the left, the selected flow's dashboard on the right. The dashboard is the flow's `metrics` section
// (sources + widgets; dxa/flow/templates.py and the rules codegen add to it): FirstRow boxes, SecondRow boxes,
// then TimeCharts. Without a selection it shows every flow's event rate side by side.
import { h, mount } from '../common/dom.js';
import { flowApi } from '../common/api.js';
import { MessageBar, Spinner, PageHeader } from '../common/components.js';
import { DataSource } from './datasource.js';
import { renderWidget, StackAreaChart } from './widgets.js';

export { DataSource, renderWidget };

export function defaultMetrics(name) {
    return {
        sources: [{
            name: 'events',
            input: { type: 'MetricApi', metricKeys: [`DATAX-${name}:Input_DataXProcessedInput_Events_Count`] },
            output: { type: 'SumWithTimeChart', data: { sum: true, timechart: true, average: true, speed: true }, dynamicOffsetInMs: 300000 }
        }, {
            name: 'latency',
            input: { type: 'MetricApi', metricKeys: [{ name: `DATAX-${name}:Latency-Process`, displayName: 'Latency-Process' },
                { name: `DATAX-${name}:Latency-Batch`, displayName: 'Latency-Batch' }] },
            output: { type: 'DirectTimeChart', data: { timechart: true }, chartTimeWindowInMs: 3600000 }
        }],
        widgets: [
            { name: 'totalEvents', displayName: 'Events ingested', data: 'events_sum', formatter: 'longint', position: 'FirstRow', type: 'SimpleBox' },
            { name: 'averageEvents', displayName: 'Avg. events / minute', data: 'events_average', formatter: 'longint', position: 'FirstRow', type: 'SimpleBox' },
            { name: 'speed', displayName: 'Current events / s', data: 'events_speed', position: 'FirstRow', type: 'Gauge' },
            { name: 'eventsChart', displayName: 'Events / second', data: 'events_timechart', position: 'TimeCharts', type: 'StackAreaChart' },
            { name: 'latencyChart', displayName: 'Batch latency (ms)', data: 'latency_timechart', position: 'TimeCharts', type: 'MultiLineChart' }
        ]
    };
}

// the dashboard of one flow; returns {root, stop}
export function Dashboard(flow, opts) {
    opts = opts || {};
    const metrics = flow.metrics && (flow.metrics.sources || []).length ? flow.metrics : defaultMetrics(flow.name);
    const vars = {};
    const root = h('div');
    const err = h('div');
    let pending = null;
    const draw = () => {
        pending = null;
        const by = pos => (metrics.widgets || []).filter(w => (w.position || 'TimeCharts') === pos).map(w => renderWidget(w, vars));
        mount(root, err,
            h('div', { class: 'dash-row' }, by('FirstRow')),
            h('div', { class: 'dash-row' }, by('SecondRow')),
            h('div', { class: 'dash-charts' }, by('TimeCharts')));
    };
    const schedule = () => {
        if (!pending) pending = setTimeout(draw, 50);
    };
    const sources = (metrics.sources || []).map(def => {
        try {
            return DataSource(def, out => { Object.assign(vars, out); schedule(); }, {
                onError: e => mount(err, MessageBar('warning', `metric source ${def.name}: ${e.message}`))
            });
        } catch (e) {
            mount(err, MessageBar('error', e.message));
            return null;
        }
    }).filter(Boolean);
    draw();
    for (const src of sources) src.start(opts.intervalMs || 5000);
    return { root, stop: () => sources.forEach(x => x.stop()) };
}

// every flow's events/s on one chart (metricAllProducts.jsx)
function AllFlows(flows, intervalMs) {
    const root = h('div');
    const def = {
        name: 'all',
        input: { type: 'MetricApi', metricKeys: flows.map(f => ({ name: `DATAX-${f.name}:Input_DataXProcessedInput_Events_Count`, displayName: f.displayName || f.name })) },
        output: { type: 'SumWithTimeChart', data: { timechart: true, sum: true }, dynamicOffsetInMs: 600000 }
    };
    const src = DataSource(def, out => mount(root, StackAreaChart({ displayName: 'Events / second, all flows' }, out.all_timechart)));
    mount(root, StackAreaChart({ displayName: 'Events / second, all flows' }, null));
    src.start(intervalMs);
    return { root, stop: () => src.stop() };
}

export function MetricExplorer(props, ctx) {
    const state = { flows: null, selected: props.name || null, error: null, interval: 5000 };
    const root = h('div');
    let active = null;

    function stopActive() {
        if (active) active.stop();
        active = null;
    }

    async function select(name) {
        stopActive();
        state.selected = name;
        if (name) history.replaceState({}, '', `/dashboard/${name}`);
        render();
        const host = root.querySelector('#dash');
        if (!name) {
            active = AllFlows(state.flows || [], state.interval);
            mount(host, active.root);
            return;
        }
        mount(host, Spinner('Loading dashboard...'));
        try {
            const flow = await flowApi.get(name);
            if (state.selected !== name) return;
            active = Dashboard(flow, { intervalMs: state.interval });
            mount(host, active.root);
        } catch (e) {
            mount(host, MessageBar('error', e.message));
        }
    }

    function render() {
        mount(
            root,
            PageHeader('Metrics',
                h('label', { class: 'row' }, 'refresh every',
                    h('select', { onchange: e => { state.interval = Number(e.target.value); select(state.selected); } },
                        [2000, 5000, 10000, 30000, 60000].map(v => h('option', { value: v, selected: v === state.interval ? true : null }, v / 1000 + ' s'))))),
            MessageBar('error', state.error),
            h('div', { class: 'cols' },
                h('div', { class: 'itemlist' },
                    h('ul', null,
                        h('li', { class: state.selected ? '' : 'on', onclick: () => select(null) }, 'All flows'),
                        (state.flows || []).map(f => h('li', { class: state.selected === f.name ? 'on' : '', onclick: () => select(f.name) }, f.displayName || f.name)))),
                h('div', { class: 'grow', id: 'dash' }))
        );
    }

    ctx.onDispose(stopActive);
    render();
    flowApi.getAllMin().then(fs => {
        state.flows = fs || [];
        select(state.selected);
    }).catch(e => {
        state.error = e.message;
        render();
    });
    return root;
}
