// Query tab with LiveQuery (datax-query: querySettingsContent.jsx, sideToolBar.jsx, kernelActions.js,
// queryActions.js). A LiveQuery kernel holds sampled input events parsed on the GPU; the selected statements (or the
// whole query) run against it and the first rows come back. Codegen preview shows the SQL the rules compile into;
// the schema preview lists the output tables' columns (userqueries/schema).
import { h, mount } from '../common/dom.js';
import { queryApi, flowApi } from '../common/api.js';
import { Button, MessageBar, Spinner, StatementBox, functionEnabled } from '../common/components.js';
import { interactiveQueryObject } from '../pipeline/inputTab.js';

export function rowsToTable(lines) {
    const rows = [];
    for (const l of lines || []) {
        try {
            rows.push(typeof l === 'string' ? JSON.parse(l) : l);
        } catch (e) {
            rows.push({ value: l });
        }
    }
    const cols = [];
    for (const r of rows) {
        if (r && typeof r === 'object' && !Array.isArray(r)) {
            for (const k of Object.keys(r)) if (!cols.includes(k)) cols.push(k);
        }
    }
    return { cols, rows };
}

function cell(v) {
    if (v === null || v === undefined) return h('span', { class: 'muted' }, 'null');
    if (typeof v === 'object') return JSON.stringify(v);
    return String(v);
}

export function ResultsTable(lines) {
    const { cols, rows } = rowsToTable(lines);
    if (!rows.length) return h('div', { class: 'muted' }, 'No rows.');
    if (!cols.length) return h('pre', { class: 'mono' }, rows.map(r => JSON.stringify(r)).join('\n'));
    return h('div', { class: 'query-results' },
        h('table', { class: 'grid compact' },
            h('thead', null, h('tr', null, cols.map(c => h('th', null, c)))),
            h('tbody', null, rows.map(r => h('tr', null, cols.map(c => h('td', null, cell(r[c]))))))));
}

export function QueryTab(flow, ui) {
    const k = ui.kernel;
    const out = h('div');
    const status = h('span', { class: 'muted' }, k.id ? `kernel ${k.id.slice(0, 8)}` : 'no kernel');
    const editor = h('textarea', {
        class: 'mono',
        style: { width: '100%', height: '300px' },
        spellcheck: 'false',
        value: flow.query,
        disabled: !functionEnabled('queryEditorEnabled'),
        oninput: e => {
            flow.query = e.target.value;
            ui.touch();
        }
    });
    const seconds = h('input', { value: '5', size: 3, title: 'seconds of input to sample' });

    const show = (...children) => mount(out, ...children);
    const busy = label => show(Spinner(label));

    async function ensureKernel() {
        if (k.id) return k.id;
        status.textContent = 'creating kernel...';
        k.id = await queryApi.createKernel(interactiveQueryObject(flow, Number(seconds.value) || 5));
        status.textContent = `kernel ${k.id.slice(0, 8)}`;
        return k.id;
    }

    async function execute() {
        const sel = editor.value.substring(editor.selectionStart, editor.selectionEnd);
        const code = sel.trim() ? sel : editor.value;
        busy('Executing on the GPU...');
        try {
            const id = await ensureKernel();
            const t0 = performance.now();
            const lines = await queryApi.executeQuery(id, code);
            k.results = lines;
            show(h('div', { class: 'muted' }, `${(lines || []).length} row(s) in ${Math.round(performance.now() - t0)} ms`), ResultsTable(lines));
        } catch (e) {
            show(MessageBar('error', e.message));
        }
    }

    async function resample() {
        busy('Sampling the input...');
        try {
            const body = interactiveQueryObject(flow, Number(seconds.value) || 5);
            if (k.id) {
                body.kernelId = k.id;
                await queryApi.refreshSampleAndKernel(body);
            } else {
                await queryApi.refreshSample(body);
                await ensureKernel();
            }
            const rows = await queryApi.sampleInput(k.id);
            show(h('div', { class: 'muted' }, 'Sampled input (first rows):'), ResultsTable(rows));
        } catch (e) {
            show(MessageBar('error', 'Resample failed: ' + e.message));
        }
    }

    async function refreshKernel() {
        busy('Refreshing the kernel...');
        try {
            if (k.id) await queryApi.deleteKernel(k.id).catch(() => null);
            k.id = null;
            await ensureKernel();
            show(MessageBar('success', 'New kernel ' + k.id.slice(0, 8)));
        } catch (e) {
            show(MessageBar('error', e.message));
        }
    }

    async function deleteAll() {
        try {
            await queryApi.deleteAllKernels();
            k.id = null;
            status.textContent = 'no kernel';
            show(MessageBar('success', 'All LiveQuery kernels deleted.'));
        } catch (e) {
            show(MessageBar('error', e.message));
        }
    }

    async function codegen() {
        busy('Generating code...');
        try {
            const cfg = await flowApi.toConfig(flow, flow.query);
            const r = await flowApi.codegen(flow.query, cfg.rules || [], flow.name);
            show(
                h('div', { class: 'panel-header' }, 'Generated query (rules compiled in)'),
                h('pre', { class: 'mono statement' }, r.code || ''),
                h('div', null, h('b', null, 'Outputs: '), (r.outputs || []).map(o => h('span', { class: 'pill' }, `${o[0]} → ${o[1]}`))),
                Object.keys(r.timeWindows || {}).length ? h('div', null, h('b', null, 'Time windows: '), JSON.stringify(r.timeWindows)) : null,
                Object.keys(r.accumulationTables || {}).length ? h('div', null, h('b', null, 'Accumulation tables: '), Object.keys(r.accumulationTables).join(', ')) : null
            );
        } catch (e) {
            show(MessageBar('error', 'Codegen failed: ' + e.message));
        }
    }

    async function schema() {
        busy('Analyzing...');
        try {
            const cfg = await flowApi.toConfig(flow, flow.query);
            const r = await flowApi.schema(flow.query, flow.input.properties.inputSchemaFile, cfg.rules || []);
            show(h('div', { class: 'panel-header' }, 'Output tables'), h('pre', { class: 'mono statement' }, JSON.stringify(r, null, 2)));
        } catch (e) {
            show(MessageBar('error', 'Schema analysis failed: ' + e.message));
        }
    }

    return h(
        'div',
        null,
        StatementBox('i', 'Statements are "Table = SELECT ...;" over DataXProcessedInput, reference data and earlier ' +
            'tables; "OUTPUT T TO <sink id>;" routes a table to an output. Select statements and Execute to run them live.'),
        editor,
        h(
            'div',
            { class: 'row' },
            Button('Execute', execute, { primary: true, disabled: !functionEnabled('executeQueryButtonEnabled') }),
            Button('Resample input', resample, { disabled: !functionEnabled('resampleButtonEnabled') }),
            h('span', null, 'for'),
            seconds,
            h('span', null, 's'),
            Button('Refresh kernel', refreshKernel, { disabled: !functionEnabled('refreshKernelsButtonEnabled') }),
            Button('Delete all kernels', deleteAll, { disabled: !functionEnabled('deleteAllKernelsEnabled') }),
            Button('Codegen preview', codegen, { disabled: !functionEnabled('previewQueryButtonEnabled') }),
            Button('Output schema', schema),
            status
        ),
        out
    );
}
