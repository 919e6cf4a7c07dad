// Flow list (datax-pipeline flowList/components/flowListPanel.jsx): every flow with its jobs' state, a filter box,
// New Flow, and links to the flow's definition and metrics dashboard.
import { h, mount } from '../common/dom.js';
import { flowApi, jobApi } from '../common/api.js';
import { PageHeader, MessageBar, Spinner, Button, functionEnabled } from '../common/components.js';

export function FlowListPanel(props, ctx) {
    const state = { flows: null, jobs: {}, filter: '', error: null };
    const root = h('div');

    function render() {
        mount(
            root,
            PageHeader(
                'Flows',
                Button('+ New Flow', () => ctx.navigate(props.newItemPath || '/config/new'), {
                    primary: true,
                    disabled: !functionEnabled('newFlowButtonEnabled')
                })
            ),
            MessageBar('error', state.error, () => { state.error = null; render(); }),
            h(
                'div',
                { class: 'panel' },
                h('input', {
                    placeholder: 'Filter by name or owner',
                    value: state.filter,
                    style: { width: '320px', marginBottom: '8px' },
                    oninput: e => {
                        state.filter = e.target.value;
                        renderRows();
                    }
                }),
                h('div', { id: 'flowrows' })
            )
        );
        renderRows();
    }

    function renderRows() {
        const host = root.querySelector('#flowrows');
        if (!host) return;
        if (state.flows === null) return mount(host, Spinner('Loading flows...'));
        const q = state.filter.trim().toLowerCase();
        const rows = state.flows.filter(f => !q || (f.displayName || '').toLowerCase().includes(q) ||
            f.name.toLowerCase().includes(q) || (f.owner || '').toLowerCase().includes(q));
        if (!rows.length) return mount(host, h('div', { class: 'muted' }, state.flows.length ? 'No flow matches the filter.' : 'No flows yet. Create one with New Flow.'));
        mount(
            host,
            h(
                'table',
                { class: 'grid' },
                h('thead', null, h('tr', null, ['Flow', 'Name', 'Owner', 'Job state', ''].map(t => h('th', null, t)))),
                h(
                    'tbody',
                    null,
                    rows.map(f => {
                        const j = state.jobs[f.name];
                        const st = j ? j.state : 'not deployed';
                        return h(
                            'tr',
                            null,
                            h('td', null, h('a', { href: `${props.editItemPath || '/config/edit'}/${f.name}`, 'data-nav': true }, f.displayName || f.name)),
                            h('td', { class: 'mono' }, f.name),
                            h('td', null, f.owner || ''),
                            h('td', { class: 'state-' + String(st).toLowerCase() }, st),
                            h('td', null, h('a', { href: `/dashboard/${f.name}`, 'data-nav': true }, 'metrics'))
                        );
                    })
                )
            )
        );
    }

    async function load() {
        try {
            const [flows, jobs] = await Promise.all([flowApi.getAllMin(), jobApi.getAll().catch(() => [])]);
            state.flows = (flows || []).sort((a, b) => (a.displayName || a.name).localeCompare(b.displayName || b.name));
            state.jobs = {};
            for (const j of jobs || []) state.jobs[j.flow || j.name] = j;
        } catch (e) {
            state.flows = [];
            state.error = e.message;
        }
        render();
    }

    render();
    load();
    return root;
}
