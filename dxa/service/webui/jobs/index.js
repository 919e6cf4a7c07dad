// Jobs page (datax-jobs components/sparkJobs.jsx, sparkJobsList.jsx; jobs/api.js): every GPU job with its state,
// GPUs, flow and links; start / stop / restart per job, Sync (job/syncall re-reads the processes' state), a state
// filter and auto-refresh.
import { h, mount } from '../common/dom.js';
import { jobApi } from '../common/api.js';
import { PageHeader, MessageBar, Spinner, Button, Toggle, functionEnabled } from '../common/components.js';

const STATES = ['all', 'running', 'idle', 'starting', 'stopping', 'error', 'success'];

export function GpuJobs(props, ctx) {
    const state = { jobs: null, filter: 'all', auto: true, error: null, info: null, busy: {} };
    const root = h('div');
    let timer = null;

    async function load() {
        try {
            state.jobs = (await jobApi.getAll()) || [];
            state.error = null;
        } catch (e) {
            state.error = e.message;
            state.jobs = state.jobs || [];
        }
        render();
    }

    async function act(name, fn, label) {
        state.busy[name] = label;
        render();
        try {
            const r = await fn(name);
            state.info = `${label} ${name}: ${r && r.state ? r.state : 'done'}`;
        } catch (e) {
            state.error = `${label} ${name} failed: ${e.message}`;
        }
        delete state.busy[name];
        await load();
    }

    function rows() {
        const js = state.jobs || [];
        return state.filter === 'all' ? js : js.filter(j => String(j.state || '').toLowerCase() === state.filter);
    }

    function render() {
        const canAct = functionEnabled('jobActionsEnabled');
        const table = state.jobs === null
            ? Spinner('Loading jobs...')
            : h('table', { class: 'grid' },
                h('thead', null, h('tr', null, ['Job', 'Flow', 'State', 'GPUs', 'App', 'Started', ''].map(t => h('th', null, t)))),
                h('tbody', null, rows().map(j => {
                    const st = String(j.state || 'unknown');
                    const busy = state.busy[j.name];
                    return h('tr', null,
                        h('td', { class: 'mono' }, j.name),
                        h('td', null, j.flow ? h('a', { href: `/config/edit/${j.flow}`, 'data-nav': true }, j.flow) : ''),
                        h('td', { class: 'state-' + st.toLowerCase() }, busy ? busy + '...' : st),
                        h('td', null, String(j.gpus || 1)),
                        h('td', null, j.app || ''),
                        h('td', null, j.startedAt ? new Date(j.startedAt * 1000).toLocaleString() : ''),
                        h('td', null,
                            h('div', { class: 'row' },
                                Button('Start', () => act(j.name, jobApi.start, 'Start'), { disabled: !canAct || !!busy || st.toLowerCase() === 'running' }),
                                Button('Stop', () => act(j.name, jobApi.stop, 'Stop'), { disabled: !canAct || !!busy || st.toLowerCase() !== 'running' }),
                                Button('Restart', () => act(j.name, jobApi.restart, 'Restart'), { disabled: !canAct || !!busy }),
                                j.flow ? h('a', { href: `/dashboard/${j.flow}`, 'data-nav': true }, 'metrics') : null)));
                })));
        mount(root,
            PageHeader('Jobs',
                h('label', { class: 'row' }, 'state',
                    h('select', { onchange: e => { state.filter = e.target.value; render(); } },
                        STATES.map(s => h('option', { value: s, selected: s === state.filter ? true : null }, s)))),
                Toggle('auto-refresh', state.auto, v => { state.auto = v; }),
                Button('Sync', async () => { await jobApi.syncAll().catch(e => (state.error = e.message)); await load(); }),
                Button('Refresh', load)),
            MessageBar('error', state.error, () => { state.error = null; render(); }),
            MessageBar('success', state.info, () => { state.info = null; render(); }),
            h('div', { class: 'panel' }, table));
    }

    const tick = async () => {
        if (state.auto) await load();
        timer = setTimeout(tick, 5000);
    };
    ctx.onDispose(() => clearTimeout(timer));
    render();
    tick();
    return root;
}
